// optim.hip — the training step that follows the rasterizer backward, for gfx950.
//
// Replaces, for the six GaussianModel parameter groups (gaussian_model.cpp:485-518):
//   * the autograd backward of the activations the renderer applies (gaussian_renderer.cpp:167-290 via
//     gaussian_model.cpp:54-77: xyz as is, cat(f_dc, f_rest), sigmoid(opacity), exp(scaling), normalize(rotation))
//   * torch::optim::Adam::step (LibTorch 2.0.1, the reference's pinned dependency, README.md:29; eps 1e-15 set at
//     gaussian_model.cpp:492) — as ~10 elementwise launches per group there, ONE launch for all groups here;
//   * addDensificationStats + the max_radii2D update (gaussian_model.cpp:839-853, gaussian_mapper.cpp:427-434);
//   * densifyAndPrune = densifyAndClone + densifyAndSplit + prunePoints (gaussian_model.cpp:700-837), as a
//     classify / scan / scatter compaction that writes the final arrays once instead of cat + index three times;
//   * resetOpacity (gaussian_model.cpp:564-592).
//
// Adam is HBM-bound streaming (per float: read p, m, v, g; write p, m, v = 28 B). Work is split into 16-B chunks
// (4 floats); each block belongs to one group, so the group's constants are wave-uniform scalar loads from the
// kernel arguments. The activation chain rule is applied to the chunk in registers (rotation chunks are exactly
// one Gaussian's quaternion), so the raw-parameter gradients never touch HBM.
//
// Float order follows LibTorch's Adam: m = m*b1 + (1-b1)*g; v = v*b2 + (1-b2)*g*g;
// p += -(lr / bc1) * m / (sqrt(v) / sqrt(bc2) + eps), bias corrections in double on the host (adam.cpp).
#include <algorithm>

#include "kernels.h"

namespace omr {

namespace {

constexpr int ADAM_THREADS = 256;
constexpr int DENSIFY_THREADS = 256;
constexpr int DENSIFY_ITEMS = 4;
constexpr int DENSIFY_TILE = DENSIFY_THREADS * DENSIFY_ITEMS;

__device__ __forceinline__ void adam_update(float& p, float& m, float& v, float g, float neg_step_size, float bc2_sqrt,
                                            float b1, float b2, float omb1, float omb2, float eps)
{
    m = fmaf(omb1, g, m * b1);
    v = fmaf(omb2 * g, g, v * b2);
    const float denom = sqrtf(v) / bc2_sqrt + eps;
    p = fmaf(neg_step_size, m / denom, p);
}

// the renderer's activations (gaussian_model.cpp:54-77) in torch's expressions: 1 / (1 + exp(-x)), exp(x),
// x / max(||x||_2, 1e-12) (F.normalize; the norm summed left to right, no contraction: -ffp-contract=off).
// activate_kernel and adam_kernel's fused outputs share them, so both give the same bits.
__device__ __forceinline__ float sigmoidf(float x) { return 1.f / (1.f + expf(-x)); }
__device__ __forceinline__ float4 normalize4(float4 q)
{
    const float d = fmaxf(sqrtf(q.x * q.x + q.y * q.y + q.z * q.z + q.w * q.w), 1e-12f);
    return make_float4(q.x / d, q.y / d, q.z / d, q.w / d);
}

// raster-gradient index of f_rest element e ([P, Mr, 3] flat) inside dL_dsh [P, M, 3], M = Mr + 1
struct RestIndex {
    uint32_t g, k, row;  // Gaussian, element within its f_rest row, f_rest row length (3 Mr)
    __device__ RestIndex(uint32_t e, uint32_t row_) : g(e / row_), k(e % row_), row(row_) {}
    __device__ uint32_t next()
    {
        const uint32_t idx = g * (row + 3) + 3 + k;
        if (++k == row) { k = 0; ++g; }
        return idx;
    }
};


// ADAM_SH_ROWS, one block: f_rest elements [E0, E1) (E0 = 1024 x block) as 16-B chunks (one per thread, float4 p / m /
// v like every other group), the f_dc elements of the Gaussians whose f_rest row starts in that range, and their
// dL_dsh / activated-SH positions, which form ONE contiguous span of the [P, M, 3] rows: the span's gradients are
// read into LDS and the updated values written back from there with lane-contiguous dword accesses (a thread reading
// its own 4 positions instead strides each wave instruction 16 B apart: 4x the transactions, and measured 44 us
// slower at 1 M Gaussians, profiles/r05l_adam_ab.txt).
constexpr int SH_SPAN_MAX = 4 * ADAM_THREADS + 3 * (4 * ADAM_THREADS / 3 + 1);  // f_rest row of 3 floats: Mr = 1
__device__ __forceinline__ void adam_sh_rows(const AdamArgs& a, const AdamGroup& G, uint32_t blk)
{
    __shared__ float s_span[SH_SPAN_MAX];
    const uint32_t R = 3u * (uint32_t)(a.M - 1), W = R + 3u;  // f_rest floats per Gaussian, dL_dsh floats per Gaussian
    const uint32_t E0 = blk * ADAM_THREADS * 4u, E1 = min(E0 + ADAM_THREADS * 4u, G.n);
    const uint32_t q0 = E0 / R, k0 = E0 - q0 * R;
    const uint32_t s0 = q0 * W + (k0 == 0u ? 0u : 3u + k0);  // the span: [s0, s1) of dL_dsh / act
    const uint32_t ql = (E1 - 1u) / R;
    const uint32_t s1 = ql * W + 3u + (E1 - 1u - ql * R) + 1u;
    const uint32_t qa = (E0 + R - 1u) / R, qb = (E1 + R - 1u) / R;  // Gaussians whose f_dc this block steps
    const uint32_t t = threadIdx.x;
    for (uint32_t i = t; i < s1 - s0; i += ADAM_THREADS) s_span[i] = G.g[s0 + i];
    __syncthreads();
    // f_rest: elements E0 + 4t .. +3
    const uint32_t e = E0 + 4u * t;
    if (e < E1) {
        const uint32_t cnt = min(4u, E1 - e);
        float p[4], m[4], v[4];
        if (cnt == 4) {
            const float4 p4 = *reinterpret_cast<const float4*>(G.p + e);
            const float4 m4 = *reinterpret_cast<const float4*>(G.m + e);
            const float4 v4 = *reinterpret_cast<const float4*>(G.v + e);
            p[0] = p4.x, p[1] = p4.y, p[2] = p4.z, p[3] = p4.w;
            m[0] = m4.x, m[1] = m4.y, m[2] = m4.z, m[3] = m4.w;
            v[0] = v4.x, v[1] = v4.y, v[2] = v4.z, v[3] = v4.w;
        } else {
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                p[j] = j < (int)cnt ? G.p[e + j] : 0.f;
                m[j] = j < (int)cnt ? G.m[e + j] : 0.f;
                v[j] = j < (int)cnt ? G.v[e + j] : 0.f;
            }
        }
        uint32_t q = e / R, k = e - q * R;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const uint32_t at = q * W + 3u + k - s0;
            if (j < (int)cnt) {
                adam_update(p[j], m[j], v[j], s_span[at], G.neg_step_size, G.bc2_sqrt, a.beta1, a.beta2, a.omb1,
                            a.omb2, a.eps);
                s_span[at] = p[j];  // the activated SH value (cat is the identity on each element)
            }
            if (++k == R) k = 0, ++q;
        }
        if (cnt == 4) {
            *reinterpret_cast<float4*>(G.p + e) = make_float4(p[0], p[1], p[2], p[3]);
            *reinterpret_cast<float4*>(G.m + e) = make_float4(m[0], m[1], m[2], m[3]);
            *reinterpret_cast<float4*>(G.v + e) = make_float4(v[0], v[1], v[2], v[3]);
        } else {
            for (uint32_t j = 0; j < cnt; ++j) G.p[e + j] = p[j], G.m[e + j] = m[j], G.v[e + j] = v[j];
        }
    }
    // f_dc of Gaussians qa .. qb-1: 3 consecutive elements each, consecutive threads
    for (uint32_t i = t; i < 3u * (qb - qa); i += ADAM_THREADS) {
        const uint32_t q = qa + i / 3u, k = i - (i / 3u) * 3u, idx = 3u * q + k;
        const uint32_t at = q * W + k - s0;
        float p = G.p2[idx], m = G.m2[idx], v = G.v2[idx];
        adam_update(p, m, v, s_span[at], G.neg_step_size2, G.bc2_sqrt2, a.beta1, a.beta2, a.omb1, a.omb2, a.eps);
        G.p2[idx] = p, G.m2[idx] = m, G.v2[idx] = v;
        s_span[at] = p;
    }
    if (!G.act) return;
    __syncthreads();
    for (uint32_t i = t; i < s1 - s0; i += ADAM_THREADS) G.act[s0 + i] = s_span[i];
}
}  // namespace

// addDensificationStats (gaussian_model.cpp:839-853) and the max_radii2D update (gaussian_mapper.cpp:427-432) for
// visibility_filter = radii > 0 (gaussian_renderer.cpp:288): one Gaussian per element
__device__ __forceinline__ void densify_stats_one(const DensifyStatsArgs& d, int i)
{
    const int r = d.radii[i];
    if (r <= 0) return;
    d.max_radii[i] = fmaxf(d.max_radii[i], (float)r);
    const float gx = d.vgrad[(size_t)i * d.vstride], gy = d.vgrad[(size_t)i * d.vstride + 1];
    d.accum[i] += sqrtf(gx * gx + gy * gy);
    d.denom[i] += 1.f;
}

// one launch over every group: blocks [a.block0[s], a.block0[s+1]) handle group s, blocks from a.stats_block0 on the
// densification statistics (4 x 256 Gaussians each, lane-contiguous)
__global__ __launch_bounds__(ADAM_THREADS) void adam_kernel(AdamArgs a)
{
    if (blockIdx.x >= a.stats_block0) {
        const int i0 = (int)((blockIdx.x - a.stats_block0) * ADAM_THREADS * 4u + threadIdx.x);
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int i = i0 + j * ADAM_THREADS;
            if (i < a.stats.P) densify_stats_one(a.stats, i);
        }
        return;
    }
    int s = 0;
#pragma unroll
    for (int k = 1; k < ADAM_MAX_GROUPS; ++k)
        if (k < a.ngroups && blockIdx.x >= a.block0[k]) s = k;
    const AdamGroup& G = a.group[s];
    if (G.kind == ADAM_SH_ROWS) {
        adam_sh_rows(a, G, blockIdx.x - a.block0[s]);
        return;
    }
    const uint32_t c = (blockIdx.x - a.block0[s]) * ADAM_THREADS + threadIdx.x;
    const uint32_t e = c * 4;  // first float of the chunk
    if (e >= G.n) return;
    const uint32_t cnt = min(4u, G.n - e);
    float p[4], m[4], v[4], g[4];
    if (cnt == 4) {
        const float4 p4 = *reinterpret_cast<const float4*>(G.p + e);
        const float4 m4 = *reinterpret_cast<const float4*>(G.m + e);
        const float4 v4 = *reinterpret_cast<const float4*>(G.v + e);
        p[0] = p4.x, p[1] = p4.y, p[2] = p4.z, p[3] = p4.w;
        m[0] = m4.x, m[1] = m4.y, m[2] = m4.z, m[3] = m4.w;
        v[0] = v4.x, v[1] = v4.y, v[2] = v4.z, v[3] = v4.w;
    } else {
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            p[j] = j < (int)cnt ? G.p[e + j] : 0.f;
            m[j] = j < (int)cnt ? G.m[e + j] : 0.f;
            v[j] = j < (int)cnt ? G.v[e + j] : 0.f;
        }
    }
    // gradient of the raw parameter
    switch (G.kind) {
    case ADAM_SH_DC: {  // f_dc element e = 3 q + k  <-  dL_dsh[q][0][k]
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const uint32_t ej = e + j, q = ej / 3u;
            g[j] = j < (int)cnt ? G.g[ej + q * 3u * (a.M - 1)] : 0.f;
        }
    } break;
    case ADAM_SH_REST: {  // f_rest element e = 3 Mr q + k  <-  dL_dsh[q][1 + k / 3][k % 3]
        RestIndex ri(e, 3u * (a.M - 1));
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const uint32_t idx = ri.next();
            g[j] = j < (int)cnt ? G.g[idx] : 0.f;
        }
    } break;
    case ADAM_ROTATION: {  // normalize backward (torch::nn::functional::normalize, eps 1e-12); n == 4P, cnt == 4
        const float4 g4 = *reinterpret_cast<const float4*>(G.g + e);
        const float gq[4] = {g4.x, g4.y, g4.z, g4.w};
        const float nrm = sqrtf(p[0] * p[0] + p[1] * p[1] + p[2] * p[2] + p[3] * p[3]);
        const float d = fmaxf(nrm, 1e-12f);
        const float dot = gq[0] * p[0] + gq[1] * p[1] + gq[2] * p[2] + gq[3] * p[3];
        const float gd = -dot / (d * d);                    // dL/d(denominator)
        const float gn = nrm >= 1e-12f ? gd / nrm : 0.f;   // through clamp_min and the 2-norm
#pragma unroll
        for (int j = 0; j < 4; ++j) g[j] = gq[j] / d + p[j] * gn;
    } break;
    default: {
        if (cnt == 4) {
            const float4 g4 = *reinterpret_cast<const float4*>(G.g + e);
            g[0] = g4.x, g[1] = g4.y, g[2] = g4.z, g[3] = g4.w;
        } else {
#pragma unroll
            for (int j = 0; j < 4; ++j) g[j] = j < (int)cnt ? G.g[e + j] : 0.f;
        }
        if (G.kind == ADAM_OPACITY) {  // sigmoid backward: g * (1 - y) * y
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const float y = sigmoidf(p[j]);
                g[j] = g[j] * (1.f - y) * y;
            }
        } else if (G.kind == ADAM_SCALING) {  // exp backward: g * exp(s)
#pragma unroll
            for (int j = 0; j < 4; ++j) g[j] = g[j] * expf(p[j]);
        }
    } break;
    }
#pragma unroll
    for (int j = 0; j < 4; ++j)
        adam_update(p[j], m[j], v[j], g[j], G.neg_step_size, G.bc2_sqrt, a.beta1, a.beta2, a.omb1, a.omb2, a.eps);
    if (cnt == 4) {
        *reinterpret_cast<float4*>(G.p + e) = make_float4(p[0], p[1], p[2], p[3]);
        *reinterpret_cast<float4*>(G.m + e) = make_float4(m[0], m[1], m[2], m[3]);
        *reinterpret_cast<float4*>(G.v + e) = make_float4(v[0], v[1], v[2], v[3]);
    } else {
        for (uint32_t j = 0; j < cnt; ++j) G.p[e + j] = p[j], G.m[e + j] = m[j], G.v[e + j] = v[j];
    }
    if (!G.act) return;
    // the next forward's input from the updated parameter (activate_kernel's expressions)
    float o[4];
    if (G.kind == ADAM_ROTATION) {  // cnt == 4: one quaternion
        const float4 r = normalize4(make_float4(p[0], p[1], p[2], p[3]));
        o[0] = r.x, o[1] = r.y, o[2] = r.z, o[3] = r.w;
    } else {
#pragma unroll
        for (int j = 0; j < 4; ++j)  // SH_DC only for Mr = 0, where the SH array is f_dc itself
            o[j] = G.kind == ADAM_OPACITY ? sigmoidf(p[j]) : (G.kind == ADAM_SH_DC ? p[j] : expf(p[j]));  // SCALING
    }
    if (cnt == 4) *reinterpret_cast<float4*>(G.act + e) = make_float4(o[0], o[1], o[2], o[3]);
    else
        for (uint32_t j = 0; j < cnt; ++j) G.act[e + j] = o[j];
}

// addDensificationStats (gaussian_model.cpp:839-853) and the max_radii2D update (gaussian_mapper.cpp:427-432)
// for visibility_filter = radii > 0 (gaussian_renderer.cpp:288)
__global__ __launch_bounds__(256) void densification_stats_kernel(int P, const int* radii, const float* vgrad,
                                                                  int vstride, float* accum, float* denom,
                                                                  float* max_radii)
{
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= P) return;
    DensifyStatsArgs d;
    d.P = P, d.radii = radii, d.vgrad = vgrad, d.vstride = vstride, d.accum = accum, d.denom = denom;
    d.max_radii = max_radii;
    densify_stats_one(d, i);
}

// ---- densifyAndPrune -----------------------------------------------------------------------------------------
// Classification of original Gaussian i (gaussian_model.cpp:812-837 with :700-810):
//   grad   = accum / denom, NaN -> 0
//   clone  = |grad| >= max_grad && max(exp(scaling)) <= percent_dense * extent   (densifyAndClone, :786-791)
//   split  =  grad  >= max_grad && max(exp(scaling)) >  percent_dense * extent   (densifyAndSplit, :741-747)
//   A clone carries grad 0 into densifyAndSplit's padded_grad and its scale is <= the bound, so clones never split.
//   prune  = sigmoid(opacity) < min_opacity || big_vs || big_ws                   (:824-833)
//            big_vs compares max_radii2D with max_screen_size, but densificationPostfix has just reset
//            max_radii2D to zeros (:730), so big_vs = 0 > max_screen_size; big_ws = max(exp(scaling)) > 0.1 extent.
//   Split copies get scaling log(exp(s) / 1.6) (:755) and are pruned on that.
// Final order (cat then mask, :719-771, :772-777, :834): [originals neither split nor pruned]
//   [clones of unpruned clone-selected, index order] [split copy 1 of each unpruned split] [split copy 2 ...]
// Flag bits: 0 keep original, 1 keep clone, 2 keep split copies, 3 split selected (indexes the normal samples).
__device__ __forceinline__ uint32_t densify_flags(int i, const float* accum, const float* denom,
                                                  const float* scaling, const float* opacity, const DensifyParams& d)
{
    float grad = accum[i] / denom[i];
    if (grad != grad) grad = 0.f;
    const float s0 = scaling[3 * i], s1 = scaling[3 * i + 1], s2 = scaling[3 * i + 2];
    const float ms = fmaxf(fmaxf(expf(s0), expf(s1)), expf(s2));
    const float bound = d.percent_dense * d.extent;
    const bool clone = fabsf(grad) >= d.max_grad && ms <= bound;
    const bool split = grad >= d.max_grad && ms > bound;
    const bool low_opacity = sigmoidf(opacity[i]) < d.min_opacity;
    const bool screen = d.max_screen_size != 0;
    const bool big_vs = screen && 0.f > (float)d.max_screen_size;
    const float ws = 0.1f * d.extent;
    const bool by_ext = screen && d.prune_by_extent;
    const bool prune = low_opacity || big_vs || (by_ext && ms > ws);
    bool prune_split = false;
    if (split) {
        const float n0 = logf(expf(s0) / 1.6f), n1 = logf(expf(s1) / 1.6f), n2 = logf(expf(s2) / 1.6f);
        const float ms2 = fmaxf(fmaxf(expf(n0), expf(n1)), expf(n2));
        prune_split = low_opacity || big_vs || (by_ext && ms2 > ws);
    }
    return (uint32_t)(!split && !prune) | (uint32_t)(clone && !prune) << 1 | (uint32_t)(split && !prune_split) << 2 |
           (uint32_t)split << 3;
}

__device__ __forceinline__ uint4 unpack_flags(uint32_t f)
{
    return make_uint4(f & 1u, (f >> 1) & 1u, (f >> 2) & 1u, (f >> 3) & 1u);
}

__device__ __forceinline__ uint4 operator+(uint4 a, uint4 b) { return make_uint4(a.x + b.x, a.y + b.y, a.z + b.z, a.w + b.w); }

// exclusive block scan of four counters at once (DENSIFY_THREADS threads)
__device__ __forceinline__ uint4 block_scan4(uint4 x, uint4* s_wave, uint4* total)
{
    const uint32_t lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    uint4 inc = x;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const uint4 y = make_uint4(__shfl_up(inc.x, o, 64), __shfl_up(inc.y, o, 64), __shfl_up(inc.z, o, 64),
                                   __shfl_up(inc.w, o, 64));
        if (lane >= (uint32_t)o) inc = inc + y;
    }
    if (lane == 63) s_wave[w] = inc;
    __syncthreads();
    uint4 off = make_uint4(0, 0, 0, 0), tot = make_uint4(0, 0, 0, 0);
#pragma unroll
    for (int k = 0; k < DENSIFY_THREADS / 64; ++k) {
        const uint4 v = s_wave[k];
        if ((uint32_t)k < w) off = off + v;
        tot = tot + v;
    }
    __syncthreads();
    *total = tot;
    return make_uint4(off.x + inc.x - x.x, off.y + inc.y - x.y, off.z + inc.z - x.z, off.w + inc.w - x.w);
}

__global__ __launch_bounds__(DENSIFY_THREADS) void densify_classify_kernel(int P, const float* accum,
                                                                           const float* denom, const float* scaling,
                                                                           const float* opacity, DensifyParams d,
                                                                           uint8_t* flags, uint4* block_sums)
{
    __shared__ uint4 s_wave[DENSIFY_THREADS / 64];
    uint4 sum = make_uint4(0, 0, 0, 0);
#pragma unroll
    for (int k = 0; k < DENSIFY_ITEMS; ++k) {
        const int i = blockIdx.x * DENSIFY_TILE + k * DENSIFY_THREADS + threadIdx.x;
        if (i < P) {
            const uint32_t f = densify_flags(i, accum, denom, scaling, opacity, d);
            flags[i] = (uint8_t)f;
            sum = sum + unpack_flags(f);
        }
    }
    uint4 total;
    block_scan4(sum, s_wave, &total);
    if (threadIdx.x == 0) block_sums[blockIdx.x] = total;
}

// exclusive scan of the nb block sums in place (one block); block_sums[nb] = totals
__global__ __launch_bounds__(DENSIFY_THREADS) void densify_scan_kernel(uint4* block_sums, uint32_t nb)
{
    __shared__ uint4 s_wave[DENSIFY_THREADS / 64];
    uint4 carry = make_uint4(0, 0, 0, 0);
    for (uint32_t base = 0; base < nb; base += DENSIFY_THREADS) {
        const uint32_t i = base + threadIdx.x;
        const uint4 x = i < nb ? block_sums[i] : make_uint4(0, 0, 0, 0);
        uint4 total;
        const uint4 ex = block_scan4(x, s_wave, &total);
        if (i < nb) block_sums[i] = carry + ex;
        carry = carry + total;
    }
    if (threadIdx.x == 0) block_sums[nb] = carry;
}

__device__ __forceinline__ void copy_row(float* dst, const float* src, int n)
{
    for (int k = 0; k < n; ++k) dst[k] = src[k];
}

__device__ __forceinline__ void zero_row(float* dst, int n)
{
    for (int k = 0; k < n; ++k) dst[k] = 0.f;
}

__global__ __launch_bounds__(DENSIFY_THREADS) void densify_scatter_kernel(int P, DensifyIO io, const uint8_t* flags,
                                                                          const uint4* block_sums, uint32_t nb)
{
    __shared__ uint4 s_wave[DENSIFY_THREADS / 64];
    const uint4 tot = block_sums[nb];  // {kept originals A, kept clones B, kept splits K, selected splits S}
    // per-thread items are contiguous (i = base + 4 t + k) so the local scan keeps index order
    const int base = blockIdx.x * DENSIFY_TILE + threadIdx.x * DENSIFY_ITEMS;
    uint32_t f[DENSIFY_ITEMS];
    uint4 sum = make_uint4(0, 0, 0, 0);
#pragma unroll
    for (int k = 0; k < DENSIFY_ITEMS; ++k) {
        f[k] = base + k < P ? flags[base + k] : 0u;
        sum = sum + unpack_flags(f[k]);
    }
    uint4 total;
    uint4 run = block_sums[blockIdx.x] + block_scan4(sum, s_wave, &total);
    const int Mr3 = 3 * io.Mr;
#pragma unroll
    for (int k = 0; k < DENSIFY_ITEMS; ++k) {
        const int i = base + k;
        const uint32_t fl = f[k];
        if (i >= P || fl == 0u) continue;
        // destinations
        int dst[4];
        int nd = 0;
        bool fresh[4];
        int split_copy[4];
        if (fl & 1u) dst[nd] = run.x, fresh[nd] = false, split_copy[nd] = -1, ++nd;
        if (fl & 2u) dst[nd] = tot.x + run.y, fresh[nd] = true, split_copy[nd] = -1, ++nd;
        if (fl & 4u) {
            dst[nd] = tot.x + tot.y + run.z, fresh[nd] = true, split_copy[nd] = 0, ++nd;
            dst[nd] = tot.x + tot.y + tot.z + run.z, fresh[nd] = true, split_copy[nd] = 1, ++nd;
        }
        // source row
        const float* x = io.p_in[0] + 3 * (size_t)i;
        const float* q = io.p_in[5] + 4 * (size_t)i;
        const float* sc = io.p_in[4] + 3 * (size_t)i;
        float R[9], s_act[3], s_new[3];
        if (fl & 4u) {  // build_rotation (general_utils.h:34-59) and the split scaling (:749-755)
            const float nq = sqrtf(q[0] * q[0] + q[1] * q[1] + q[2] * q[2] + q[3] * q[3]);
            const float r = q[0] / nq, qx = q[1] / nq, qy = q[2] / nq, qz = q[3] / nq;
            R[0] = 1.f - 2.f * (qy * qy + qz * qz), R[1] = 2.f * (qx * qy - r * qz), R[2] = 2.f * (qx * qz + r * qy);
            R[3] = 2.f * (qx * qy + r * qz), R[4] = 1.f - 2.f * (qx * qx + qz * qz), R[5] = 2.f * (qy * qz - r * qx);
            R[6] = 2.f * (qx * qz - r * qy), R[7] = 2.f * (qy * qz + r * qx), R[8] = 1.f - 2.f * (qx * qx + qy * qy);
            for (int c = 0; c < 3; ++c) s_act[c] = expf(sc[c]), s_new[c] = logf(s_act[c] / 1.6f);
        }
        for (int t = 0; t < nd; ++t) {
            const size_t o = (size_t)dst[t];
            // xyz
            if (split_copy[t] >= 0) {
                const float* z = io.normals + 3 * ((size_t)split_copy[t] * tot.w + run.w);
                const float sm[3] = {z[0] * s_act[0], z[1] * s_act[1], z[2] * s_act[2]};
                for (int r = 0; r < 3; ++r)
                    io.p_out[0][3 * o + r] = R[3 * r] * sm[0] + R[3 * r + 1] * sm[1] + R[3 * r + 2] * sm[2] + x[r];
            } else {
                copy_row(io.p_out[0] + 3 * o, x, 3);
            }
            copy_row(io.p_out[1] + 3 * o, io.p_in[1] + 3 * (size_t)i, 3);
            copy_row(io.p_out[2] + Mr3 * o, io.p_in[2] + Mr3 * (size_t)i, Mr3);
            io.p_out[3][o] = io.p_in[3][i];
            if (split_copy[t] >= 0) copy_row(io.p_out[4] + 3 * o, s_new, 3);
            else copy_row(io.p_out[4] + 3 * o, sc, 3);
            copy_row(io.p_out[5] + 4 * o, q, 4);
            if (io.exist_out) io.exist_out[o] = io.exist_in[i];
            // optimizer state: moved with the point, zeros for new points (:702-716)
            const int width[6] = {3, 3, Mr3, 1, 3, 4};
            for (int gidx = 0; gidx < 6; ++gidx) {
                const int w = width[gidx];
                if (io.m_out[gidx]) {
                    if (fresh[t] || !io.m_in[gidx]) zero_row(io.m_out[gidx] + w * o, w);
                    else copy_row(io.m_out[gidx] + w * o, io.m_in[gidx] + w * (size_t)i, w);
                }
                if (io.v_out[gidx]) {
                    if (fresh[t] || !io.v_in[gidx]) zero_row(io.v_out[gidx] + w * o, w);
                    else copy_row(io.v_out[gidx] + w * o, io.v_in[gidx] + w * (size_t)i, w);
                }
            }
        }
        run = run + unpack_flags(fl);
    }
}

// resetOpacity (gaussian_model.cpp:564-572): opacity = inverse_sigmoid(min(sigmoid(opacity), ceiling)), moments 0
__global__ __launch_bounds__(256) void reset_opacity_kernel(int P, float* opacity, float* m, float* v, float ceiling)
{
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= P) return;
    const float x = fminf(sigmoidf(opacity[i]), ceiling);
    opacity[i] = logf(x / (1.f - x));
    if (m) m[i] = 0.f;
    if (v) v[i] = 0.f;
}

// ---- the activations of the renderer (gaussian_model.cpp:54-77, gaussian_renderer.cpp:175-200) --------------------
// One launch instead of torch's cat + sigmoid + exp + normalize (six launches, 0.20 ms at config C in
// profiles/r05e_train_kernel_stats.csv): blocks [0, sh_blocks) copy cat(f_dc, f_rest) into the [P, Mr + 1, 3] SH
// array the rasterizer reads (16 B of output per thread, gathered from the two inputs), the rest apply sigmoid /
// exp / normalize per Gaussian (sigmoidf, expf, normalize4 above). In the training loop Adam writes these outputs
// itself (AdamGroup::act) and this launch runs only when the parameters changed outside Adam.
constexpr int ACT_THREADS = 256;
__global__ __launch_bounds__(ACT_THREADS) void activate_kernel(ActivateArgs a, uint32_t sh_blocks)
{
    if (blockIdx.x < sh_blocks) {  // 32-bit indices: P * 3 (Mr + 1) < 2^32 (omr_activate)
        const uint32_t row = 3u * (uint32_t)(a.Mr + 1);  // floats per Gaussian in the output
        const uint32_t n = (uint32_t)a.P * row;
        const uint32_t e0 = (blockIdx.x * ACT_THREADS + threadIdx.x) * 4u;
        if (e0 >= n) return;
        uint32_t g = e0 / row, k = e0 - g * row;
        float o[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            o[j] = e0 + j >= n ? 0.f : (k < 3u ? a.f_dc[3u * g + k] : a.f_rest[g * (row - 3u) + (k - 3u)]);
            if (++k == row) k = 0, ++g;
        }
        if (e0 + 4u <= n) *reinterpret_cast<float4*>(a.shs + e0) = make_float4(o[0], o[1], o[2], o[3]);
        else
            for (uint32_t j = 0; j < 4u && e0 + j < n; ++j) a.shs[e0 + j] = o[j];
        return;
    }
    const uint32_t i = (blockIdx.x - sh_blocks) * ACT_THREADS + threadIdx.x;
    if (i >= (uint32_t)a.P) return;
    a.opacity_out[i] = sigmoidf(a.opacity[i]);
#pragma unroll
    for (int c = 0; c < 3; ++c) a.scales_out[3 * i + c] = expf(a.scaling[3 * i + c]);
    *reinterpret_cast<float4*>(a.rotations_out + 4 * (size_t)i) =
        normalize4(*reinterpret_cast<const float4*>(a.rotation + 4 * (size_t)i));
}

// ---- launchers -------------------------------------------------------------------------------------------------
void launch_activate(const ActivateArgs& a, hipStream_t s)
{
    if (a.P <= 0) return;
    const uint32_t sh_blocks =
        a.shs ? (uint32_t)div_up(div_up((size_t)a.P * 3 * (a.Mr + 1), (size_t)4), (size_t)ACT_THREADS) : 0u;
    // opacity_out NULL: the SH copy alone (omr_adam_step_activate without the SH row walk)
    const uint32_t blocks = sh_blocks + (a.opacity_out ? div_up((uint32_t)a.P, (uint32_t)ACT_THREADS) : 0u);
    if (blocks == 0) return;
    activate_kernel<<<blocks, ACT_THREADS, 0, s>>>(a, sh_blocks);
}

void launch_adam(AdamArgs a, hipStream_t s)
{
    uint32_t blocks = 0;
    for (int k = 0; k < a.ngroups; ++k) {
        a.block0[k] = blocks;
        blocks += div_up(div_up(a.group[k].n, 4u), (uint32_t)ADAM_THREADS);
    }
    for (int k = a.ngroups; k < ADAM_MAX_GROUPS; ++k) a.block0[k] = blocks;
    a.stats_block0 = blocks;
    if (a.stats.P > 0) blocks += div_up((uint32_t)a.stats.P, 4u * ADAM_THREADS);
    if (blocks) adam_kernel<<<blocks, ADAM_THREADS, 0, s>>>(a);
}

void launch_densification_stats(int P, const int* radii, const float* vgrad, int vstride, float* accum, float* denom,
                                float* max_radii, hipStream_t s)
{
    if (P > 0)
        densification_stats_kernel<<<div_up((uint32_t)P, 256u), 256, 0, s>>>(P, radii, vgrad, vstride, accum, denom,
                                                                             max_radii);
}

size_t densify_plan_bytes(int P)
{
    const size_t nb = div_up((size_t)std::max(P, 0), (size_t)DENSIFY_TILE);
    return align_up((size_t)std::max(P, 0)) + (nb + 1) * sizeof(uint4);
}

void launch_densify_plan(int P, const float* accum, const float* denom, const float* scaling, const float* opacity,
                         float max_grad, float min_opacity, float extent, float percent_dense, int max_screen_size,
                         int prune_by_extent, char* plan, hipStream_t s)
{
    const uint32_t nb = div_up((uint32_t)std::max(P, 0), (uint32_t)DENSIFY_TILE);
    uint8_t* flags = reinterpret_cast<uint8_t*>(plan);
    uint4* sums = reinterpret_cast<uint4*>(plan + align_up((size_t)std::max(P, 0)));
    const DensifyParams d{max_grad, min_opacity, extent, percent_dense, max_screen_size, prune_by_extent};
    if (nb) densify_classify_kernel<<<nb, DENSIFY_THREADS, 0, s>>>(P, accum, denom, scaling, opacity, d, flags, sums);
    densify_scan_kernel<<<1, DENSIFY_THREADS, 0, s>>>(sums, nb);
}

const uint4* densify_plan_totals(int P, const char* plan)
{
    const uint32_t nb = div_up((uint32_t)std::max(P, 0), (uint32_t)DENSIFY_TILE);
    return reinterpret_cast<const uint4*>(plan + align_up((size_t)std::max(P, 0))) + nb;
}

void launch_densify_apply(int P, const char* plan, const DensifyIO& io, hipStream_t s)
{
    const uint32_t nb = div_up((uint32_t)std::max(P, 0), (uint32_t)DENSIFY_TILE);
    if (!nb) return;
    const uint8_t* flags = reinterpret_cast<const uint8_t*>(plan);
    const uint4* sums = reinterpret_cast<const uint4*>(plan + align_up((size_t)P));
    densify_scatter_kernel<<<nb, DENSIFY_THREADS, 0, s>>>(P, io, flags, sums, nb);
}

void launch_reset_opacity(int P, float* opacity, float* m, float* v, float ceiling, hipStream_t s)
{
    if (P > 0) reset_opacity_kernel<<<div_up((uint32_t)P, 256u), 256, 0, s>>>(P, opacity, m, v, ceiling);
}

}  // namespace omr
