// wave_ops.h — wave64 cross-lane reductions for gfx950 (DPP, v_permlane{16,32}_swap, LDS transposition).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace omr {

// v + (value of lane given by the DPP control); bound_ctrl: out-of-row sources read 0
template <int CTRL>
__device__ __forceinline__ float add_dpp(float keep, float send)
{
    return keep + __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, send), CTRL, 0xf, 0xf, true));
}
constexpr int DPP_XOR1 = 0xb1;   // quad_perm [1,0,3,2]
constexpr int DPP_XOR2 = 0x4e;   // quad_perm [2,3,0,1]
constexpr int DPP_ROR4 = 0x124;  // row_ror:4
constexpr int DPP_ROR8 = 0x128;  // row_ror:8
constexpr int DPP_HALF_MIRROR = 0x141;  // row_half_mirror: lane i <-> 7 - i within each 8 lanes

// Sum over the four 16-lane rows: x(lane) + x(lane^16) + x(lane^32) + x(lane^48). v_permlane16_swap swaps the
// odd rows of its first operand with the even rows of its second; with both operands = x, vdst' + src' =
// own + partner on every lane (likewise v_permlane32_swap for the two halves). Inline asm: ROCm 7.2 folds
// __builtin_amdgcn_permlane16_swap(x, x) into "2 * first result" (seen in the .s), which is wrong. The
// s_nop 1 covers the VALU-write -> permlane-read hazard, which hipcc does not pad inside asm.
__device__ __forceinline__ float cross_row_sum(float x)
{
    float a = x, b = x;
    asm volatile("s_nop 1\n\tv_permlane16_swap_b32 %0, %1" : "+v"(a), "+v"(b));
    x = a + b;
    a = x;
    b = x;
    asm volatile("s_nop 1\n\tv_permlane32_swap_b32 %0, %1" : "+v"(a), "+v"(b));
    return a + b;
}

// Wave-sum of v[0..7] and v8 with the cross-row levels FIRST, where v_permlane32_swap / v_permlane16_swap move
// whole halves / rows between two registers in one instruction (no per-lane select, unlike the DPP levels):
//   level 1  permlane32_swap(v[i], v[i+4]) + add: lanes 0-31 hold v[i] summed with lane+32, lanes 32-63 v[i+4]
//   level 2  permlane16_swap(a[i], a[i+2]) + add: row r of b[i] holds value index i + 2r, summed over 4 rows
//   level 3  within the row (DPP row_ror:8, select by lane bit 3), then an 8-lane sum (xor1, xor2, half mirror)
// 26 VALU (+2 s_nop) against 34 for a transposed DPP butterfly. Returns, in every lane l, the wave total of value index
// (l >> 3) & 7; *t8 = the total of v8 on every lane.
__device__ __forceinline__ float wave_sum9_rows(const float v[8], float v8, uint32_t lane, float* t8)
{
    float x0 = v[0], x1 = v[1], x2 = v[2], x3 = v[3], y0 = v[4], y1 = v[5], y2 = v[6], y3 = v[7], w0 = v8, w1 = v8;
    asm volatile("s_nop 1\n\t"
                 "v_permlane32_swap_b32 %0, %4\n\t"
                 "v_permlane32_swap_b32 %1, %5\n\t"
                 "v_permlane32_swap_b32 %2, %6\n\t"
                 "v_permlane32_swap_b32 %3, %7\n\t"
                 "v_permlane32_swap_b32 %8, %9"
                 : "+v"(x0), "+v"(x1), "+v"(x2), "+v"(x3), "+v"(y0), "+v"(y1), "+v"(y2), "+v"(y3), "+v"(w0), "+v"(w1));
    float a0 = x0 + y0, a1 = x1 + y1, a2 = x2 + y2, a3 = x3 + y3, u0 = w0 + w1, u1 = u0;
    asm volatile("s_nop 1\n\t"
                 "v_permlane16_swap_b32 %0, %2\n\t"
                 "v_permlane16_swap_b32 %1, %3\n\t"
                 "v_permlane16_swap_b32 %4, %5"
                 : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(u0), "+v"(u1));
    const float b0 = a0 + a2, b1 = a1 + a3;  // row r: index 2r (b0) and 2r + 1 (b1), 4 rows summed
    float u = u0 + u1;
    const bool hi = lane & 8;
    float c = add_dpp<DPP_ROR8>(hi ? b1 : b0, hi ? b0 : b1);
    c = add_dpp<DPP_XOR1>(c, c);
    c = add_dpp<DPP_XOR2>(c, c);
    c = add_dpp<DPP_HALF_MIRROR>(c, c);
    u = add_dpp<DPP_ROR8>(u, u);
    u = add_dpp<DPP_XOR1>(u, u);
    u = add_dpp<DPP_XOR2>(u, u);
    *t8 = add_dpp<DPP_HALF_MIRROR>(u, u);
    return c;
}

// Wave-sum of v[0..7] through LDS, v8 through permlane/DPP. s_red: this wave's float[8 * WS_LDS_STRIDE]. Each lane
// writes its eight values to the eight rows; lane l then adds the 8 entries (l & 7) * 8 .. + 7 of row l >> 3 (two
// 16-B reads) and the 8 lanes of a row group combine by DPP: 7 adds + 3 DPP + 8 for v8 = 18 VALU (26 for
// wave_sum9_rows), the transposition done by the LDS pipe. Same result layout as wave_sum9_rows: lane l holds the
// total of value (l >> 3) & 7, *t8 = the total of v8 on every lane. The caller orders the LDS accesses (wave_sync).
constexpr int WS_LDS_STRIDE = 68;  // floats per row: 16-B aligned rows, row starts on different banks
__device__ __forceinline__ float wave_sum9_lds(const float v[8], float v8, uint32_t lane, float* s_red, float* t8)
{
#pragma unroll
    for (int k = 0; k < 8; ++k) s_red[k * WS_LDS_STRIDE + lane] = v[k];
    float u0 = v8, u1 = v8;
    asm volatile("s_nop 1\n\tv_permlane32_swap_b32 %0, %1" : "+v"(u0), "+v"(u1));
    float u = u0 + u1;
    u0 = u;
    u1 = u;
    asm volatile("s_nop 1\n\tv_permlane16_swap_b32 %0, %1" : "+v"(u0), "+v"(u1));
    u = u0 + u1;
    u = add_dpp<DPP_ROR8>(u, u);
    u = add_dpp<DPP_XOR1>(u, u);
    u = add_dpp<DPP_XOR2>(u, u);
    *t8 = add_dpp<DPP_HALF_MIRROR>(u, u);
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    const float4* seg = reinterpret_cast<const float4*>(s_red + (lane >> 3) * WS_LDS_STRIDE + (lane & 7) * 8);
    const float4 a = seg[0], b = seg[1];
    float c = ((a.x + a.y) + (a.z + a.w)) + ((b.x + b.y) + (b.z + b.w));
    c = add_dpp<DPP_XOR1>(c, c);
    c = add_dpp<DPP_XOR2>(c, c);
    return add_dpp<DPP_HALF_MIRROR>(c, c);
}

// Wave-sums of two instances' nine values, the first eight of each already stored by the caller: a's in rows 0-7 of
// s_red (float[16 * WS_LDS_STRIDE]), b's in rows 8-15 (row k, lane l at k * WS_LDS_STRIDE + l). Lane l sums 16
// consecutive partials of value l >> 2 and two DPP steps finish the 4-lane groups, so lane 4k returns value k
// (k < 8: a's, k >= 8: b's). The 9th values share one permlane/DPP chain: v_permlane32_swap with a in the first
// operand and b in the second leaves a's pair sums in lanes 0-31 and b's in 32-63, and the rest of the chain stays
// inside each half, so *t8 = sum a8 on lanes 0-31 and sum b8 on lanes 32-63.
__device__ __forceinline__ float wave_sum9x2_stored(float va8, float vb8, uint32_t lane, const float* s_red, float* t8)
{
    float u0 = va8, u1 = vb8;
    asm volatile("s_nop 1\n\tv_permlane32_swap_b32 %0, %1" : "+v"(u0), "+v"(u1));
    float u = u0 + u1;
    u0 = u;
    u1 = u;
    asm volatile("s_nop 1\n\tv_permlane16_swap_b32 %0, %1" : "+v"(u0), "+v"(u1));
    u = u0 + u1;
    u = add_dpp<DPP_ROR8>(u, u);
    u = add_dpp<DPP_XOR1>(u, u);
    u = add_dpp<DPP_XOR2>(u, u);
    *t8 = add_dpp<DPP_HALF_MIRROR>(u, u);
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    const float4* seg = reinterpret_cast<const float4*>(s_red + (lane >> 2) * WS_LDS_STRIDE + (lane & 3) * 16);
    const float4 a = seg[0], b = seg[1], c = seg[2], d = seg[3];
    float s = (((a.x + a.y) + (a.z + a.w)) + ((b.x + b.y) + (b.z + b.w))) +
              (((c.x + c.y) + (c.z + c.w)) + ((d.x + d.y) + (d.z + d.w)));
    s = add_dpp<DPP_XOR1>(s, s);
    return add_dpp<DPP_XOR2>(s, s);
}

}  // namespace omr
