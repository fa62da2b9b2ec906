// band_lists.h — per-wave compaction of a staged batch of tile instances (render_fwd.hip, render_bwd.hip).
//
// A tile workgroup is four wave64s, wave b owning the 16x4-pixel band b of the 16x16 tile. Each staged
// instance carries band_mask (raster_common.h): the bands its alpha >= 1/255 ellipse can reach. Instead of
// every wave testing every instance (a uniform branch and its scalar bookkeeping per instance), the batch
// is compacted once into four ordered index lists, one per band; wave b then walks only list b. Order is
// preserved (ballot ranks within a wave, per-wave counts across waves), so every pixel still visits its
// instances in the reference's front-to-back (or back-to-front) order.
#pragma once

#include "raster_common.h"

namespace omr {

template <int N>  // batch entries, staged by threads t < N (N a multiple of 64, at most 256)
struct BandLists {
    static_assert(N % 64 == 0 && N <= 256, "batch");
    static constexpr int Q = N / 64;  // staging waves
    uint8_t idx[4][N];                // idx[b][k]: batch index of the k-th instance reaching band b
    uint32_t wcnt[4][Q];              // per band, per staging wave: instances reaching the band

    // every thread of the block calls this (it holds __syncthreads); m = band mask of entry t (0 if t >= N
    // or the entry is empty)
    __device__ __forceinline__ void build(uint32_t m, uint32_t t)
    {
        const uint32_t w = t >> 6;
        uint32_t rank[4];
        if (t < (uint32_t)N) {  // wave-uniform
#pragma unroll
            for (int b = 0; b < 4; ++b) {
                const uint64_t bal = __ballot((m >> b) & 1u);
                rank[b] = mask_rank(bal);
                if ((t & 63) == 0) wcnt[b][w] = (uint32_t)__popcll(bal);
            }
        }
        __syncthreads();
        if (t < (uint32_t)N) {
#pragma unroll
            for (int b = 0; b < 4; ++b) {
                if ((m >> b) & 1u) {
                    uint32_t off = 0;
#pragma unroll
                    for (int q = 0; q < Q; ++q) off += (uint32_t)q < w ? wcnt[b][q] : 0u;
                    idx[b][off + rank[b]] = (uint8_t)t;
                }
            }
        }
        __syncthreads();
    }

    __device__ __forceinline__ uint32_t count(uint32_t b) const
    {
        uint32_t c = 0;
#pragma unroll
        for (int q = 0; q < Q; ++q) c += wcnt[b][q];
        return c;
    }
};

}  // namespace omr
