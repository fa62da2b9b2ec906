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

// wave_rows_load in two halves: wave_rows_fetch issues the NF4 loads into registers (the same lane-contiguous spans
// and the same src[0] stand-in outside the selection) without waiting for them; wave_rows_park later moves them into
// the LDS image. Between the two the wave does other work while the loads are in flight.
// the registers of an in-flight row span: native vectors (an array of float4 — HIP's struct vector type — held
// across other code is kept in scratch memory by the compiler)
typedef float rowv4 __attribute__((ext_vector_type(4)));
template <int NF4>
__device__ __forceinline__ void wave_rows_fetch(const float4* __restrict__ src, uint64_t rows, int ncols, uint32_t lane,
                                                rowv4 (&v)[NF4])
{
    const rowv4* s = reinterpret_cast<const rowv4*>(src);
#pragma unroll
    for (int q = 0; q < NF4; ++q) {
        const uint32_t k = (uint32_t)q * 64u + lane;
        const uint32_t r = k / NF4, c = k - r * NF4;
        const bool ok = ((rows >> r) & 1u) && (int)c < ncols;
        v[q] = s[ok ? k : 0u];
    }
}
template <int NF4>
__device__ __forceinline__ void wave_rows_park(const rowv4 (&v)[NF4], float4* lds, uint32_t lane)
{
    constexpr int S = stage_stride<NF4>();
#pragma unroll
    for (int q = 0; q < NF4; ++q) {
        const uint32_t k = (uint32_t)q * 64u + lane;
        const uint32_t r = k / NF4, c = k - r * NF4;
        reinterpret_cast<rowv4*>(lds)[r * S + c] = v[q];
    }
}

// Rows r with bit r of `rows` set: lds[r*S + c] -> global dst[r*NF4 + c], all NF4 columns.
template <int NF4>
__device__ __forceinline__ void wave_rows_store(float4* __restrict__ dst, uint64_t rows, const float4* lds,
                                                uint32_t lane)
{
    constexpr int S = stage_stride<NF4>();
    // every LDS read first, into registers of their own, then the stores: a store reads its data registers after it
    // issues, so refilling one register quad per store made each store wait (vmcnt) for the one before it
    rowv4 v[NF4];
#pragma unroll
    for (int q = 0; q < NF4; ++q) {
        const uint32_t k = (uint32_t)q * 64u + lane;
        const uint32_t r = k / NF4, c = k - r * NF4;
        v[q] = reinterpret_cast<const rowv4*>(lds)[r * S + c];
    }
#pragma unroll
    for (int q = 0; q < NF4; ++q) {
        const uint32_t k = (uint32_t)q * 64u + lane;
        const uint32_t r = k / NF4;
        if ((rows >> r) & 1u) reinterpret_cast<rowv4*>(dst)[k] = v[q];
    }
}

}  // namespace omr
