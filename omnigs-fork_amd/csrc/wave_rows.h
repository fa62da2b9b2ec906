// wave_rows.h — wave-cooperative staging of per-Gaussian rows through LDS (preprocess.hip, gaussian_bwd.hip).
//
// One thread per Gaussian wants its own row of a [P][NF4] float4 array (the 192-B SH row, the 64-B render record).
// Read or written lane by lane, every wave-instruction touches 64 rows NF4*16 B apart: 64 distinct cache lines
// per instruction, the address path (not HBM) sets the rate, and SQ counters show ~55-70 % of the wave cycles
// stalled on instruction issue (profiles/r01h_sq.csv). Staged, the wave moves its 64 rows as one contiguous
// 64*NF4*16-B span: instruction q of lane l carries float4 q*64+l (1 KiB contiguous per instruction), parked in
// LDS, and each lane then reads / writes its own row there.
//
// LDS image: row r at float4 r*S, S = NF4 | 1 (odd): the 16 lanes of one ds_read_b128 lane group reach 16
// distinct 4-bank groups of the 64 banks (MI355X_MICROARCH.md, LDS), so the per-lane row reads are conflict-free.
// Only the calling wave touches its image; wave_sync() (tile_wave.h) orders the phases.
#pragma once

#include "tile_wave.h"

namespace omr {

template <int NF4>
constexpr int stage_stride()
{
    return NF4 | 1;
}

// LDS float4s a wave needs to stage 64 rows of NF4 float4
template <int NF4>
constexpr int stage_f4()
{
    return 64 * stage_stride<NF4>();
}

// Rows r with bit r of `rows` set, columns [0, ncols): global src[r*NF4 + c] -> lds[r*S + c]. Branch-free: a
// float4 outside the selection reads src[0] instead (the wave's first row, which exists; one broadcast line) and
// lands in its LDS slot as a value no reader uses, so all NF4 loads are in flight before the first LDS store.
// Rows outside `rows` and columns >= ncols of the image hold garbage afterwards.
template <int NF4>
__device__ __forceinline__ void wave_rows_load(const float4* __restrict__ src, uint64_t rows, int ncols, float4* lds,
                                               uint32_t lane)
{
    constexpr int S = stage_stride<NF4>();
    float4 v[NF4];
#pragma unroll
    for (int q = 0; q < NF4; ++q) {
        const uint32_t k = (uint32_t)q * 64u + lane;
        const uint32_t r = k / NF4, c = k - r * NF4;
        const bool ok = ((rows >> r) & 1u) && (int)c < ncols;
        v[q] = src[ok ? k : 0u];
    }
#pragma unroll
    for (int q = 0; q < NF4; ++q) {
        const uint32_t k = (uint32_t)q * 64u + lane;
        const uint32_t r = k / NF4, c = k - r * NF4;
        lds[r * S + c] = v[q];
    }
}

// Rows r with bit r of `rows` set: lds[r*S + c] -> global dst[r*NF4 + c], all NF4 columns.
template <int NF4>
__device__ __forceinline__ void wave_rows_store(float4* __restrict__ dst, uint64_t rows, const float4* lds,
                                                uint32_t lane)
{
    constexpr int S = stage_stride<NF4>();
#pragma unroll
    for (int q = 0; q < NF4; ++q) {
        const uint32_t k = (uint32_t)q * 64u + lane;
        const uint32_t r = k / NF4, c = k - r * NF4;
        if ((rows >> r) & 1u) dst[k] = lds[r * S + c];
    }
}

// LDS-DMA staging (global_load_lds_dwordx4, gfx950): columns [C0, C0 + NC) of the 64 rows go straight from HBM to
// LDS, no VGPR holds them. One DMA wave-instruction writes 64 consecutive float4 of LDS (lane l -> base + 16 l), so
// the odd row stride of the image (S = NC | 1: conflict-free per-lane row reads, as above) is made on the SOURCE side:
// LDS position p = q * 64 + lane holds row p / S, column p % S; a padding slot (column NC) or an unselected row loads
// src[0] (a line the wave reads anyway) and lands where no reader looks. S instructions per call. The caller waits with
// dma_wait() and orders with wave_sync() before reading the image.
template <int NC>
constexpr int dma_stride()
{
    return NC | 1;
}
template <int NF4, int C0, int NC>
__device__ __forceinline__ void wave_rows_dma(const float4* __restrict__ src, uint64_t rows, int ncols, float4* lds,
                                              uint32_t lane)
{
    constexpr int S = dma_stride<NC>();
#pragma unroll
    for (int q = 0; q < S; ++q) {
        const uint32_t p = (uint32_t)q * 64u + lane;
        const uint32_t r = p / S, c = p - r * S;
        const bool ok = (c < (uint32_t)NC) & (((rows >> r) & 1u) != 0) & ((int)(C0 + c) < ncols);  // branch-free
        __builtin_amdgcn_global_load_lds(src + (ok ? r * NF4 + C0 + c : 0u), lds + q * 64, 16, 0, 0);
    }
}
// every LDS-DMA of the wave has landed (they count in vmcnt with the wave's other vector-memory operations)
__device__ __forceinline__ void dma_wait() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }

}  // namespace omr
