// knn.hip — distCUDA2 for gfx950: the mean squared distance of every point to its 3 nearest other points
// (third_party/simple-knn/spatial.cu:15-25, simple_knn.cu:185-220), which GaussianModel uses to initialise
// scales (gaussian_model.cpp:161, :243, :330).
//
// The reference sorts the points by a 30-bit Morton code, cuts the sorted order into boxes of 1024, seeds each
// query's rejection radius with its +-3 sorted neighbours, and scans every box whose bounding-box distance passes
// that radius and the running 3rd-best (simple_knn.cu:145-183). Box pruning only drops points that cannot be
// among the 3 nearest, so the result is the exact 3-NN mean. We keep that result and re-cut the work for wave64:
//   * the same Morton codes (10 bits per axis over the bounds of the points AND the origin: the reference's
//     reduction starts from {0,0,0}, simple_knn.cu:189) sorted with our stable LSD radix sort (sort.hip);
//   * boxes of 64 sorted points (one wave) grouped into superboxes of 64 boxes (4096 points);
//   * one wave per box of 64 queries: a superbox, then a box, is visited when ANY lane's box distance passes
//     its bound (wave ballot, no barriers); a visited box's 64 points are staged in LDS by the wave and every
//     lane scans them. Bounds are wave-uniform scalar loads.
// Squared distances are dx*dx + dy*dy + dz*dz without contraction (this file builds with -ffp-contract=off), the
// kept minima are exact, so results are bit-exact against the float32 brute-force oracle.
#include <cfloat>

#include "kernels.h"
#include "tile_wave.h"

namespace omr {

namespace {

constexpr int KNN_BOX = 64;
constexpr int KNN_SUPER = 64;  // boxes per superbox
constexpr int BOUNDS_THREADS = 256;
constexpr int BOUNDS_BLOCKS = 256;

struct Bounds {
    float4 mn, mx;
};

__device__ __forceinline__ uint32_t prep_morton(uint32_t x)
{
    x = (x | (x << 16)) & 0x030000FF;
    x = (x | (x << 8)) & 0x0300F00F;
    x = (x | (x << 4)) & 0x030C30C3;
    x = (x | (x << 2)) & 0x09249249;
    return x;
}

__device__ __forceinline__ float box_dist(const Bounds& b, float px, float py, float pz)
{
    float dx = 0.f, dy = 0.f, dz = 0.f;
    if (px < b.mn.x || px > b.mx.x) dx = fminf(fabsf(px - b.mn.x), fabsf(px - b.mx.x));
    if (py < b.mn.y || py > b.mx.y) dy = fminf(fabsf(py - b.mn.y), fabsf(py - b.mx.y));
    if (pz < b.mn.z || pz > b.mx.z) dz = fminf(fabsf(pz - b.mn.z), fabsf(pz - b.mx.z));
    return dx * dx + dy * dy + dz * dz;
}

__device__ __forceinline__ void update_best(float d, float& b0, float& b1, float& b2)
{
    // insertion into the ascending triple (simple_knn.cu:131-143 keeps the same three values)
    if (d < b2) {
        if (d < b1) {
            b2 = b1;
            if (d < b0) b1 = b0, b0 = d;
            else b1 = d;
        } else {
            b2 = d;
        }
    }
}

__device__ __forceinline__ float sqdist(float ax, float ay, float az, float bx, float by, float bz)
{
    const float dx = bx - ax, dy = by - ay, dz = bz - az;
    return dx * dx + dy * dy + dz * dz;
}

}  // namespace

// partial min / max of the points; block 0's slot also folds in the origin (the reference's reduction init)
__global__ __launch_bounds__(BOUNDS_THREADS) void knn_bounds_kernel(int P, const float* pts, Bounds* partial)
{
    __shared__ Bounds s[BOUNDS_THREADS];
    float4 mn = make_float4(0.f, 0.f, 0.f, 0.f), mx = mn;  // origin included
    for (int i = blockIdx.x * BOUNDS_THREADS + threadIdx.x; i < P; i += gridDim.x * BOUNDS_THREADS) {
        const float x = pts[3 * i], y = pts[3 * i + 1], z = pts[3 * i + 2];
        mn.x = fminf(mn.x, x), mn.y = fminf(mn.y, y), mn.z = fminf(mn.z, z);
        mx.x = fmaxf(mx.x, x), mx.y = fmaxf(mx.y, y), mx.z = fmaxf(mx.z, z);
    }
    s[threadIdx.x] = {mn, mx};
    __syncthreads();
    for (int o = BOUNDS_THREADS / 2; o > 0; o >>= 1) {
        if ((int)threadIdx.x < o) {
            Bounds a = s[threadIdx.x];
            const Bounds b = s[threadIdx.x + o];
            a.mn.x = fminf(a.mn.x, b.mn.x), a.mn.y = fminf(a.mn.y, b.mn.y), a.mn.z = fminf(a.mn.z, b.mn.z);
            a.mx.x = fmaxf(a.mx.x, b.mx.x), a.mx.y = fmaxf(a.mx.y, b.mx.y), a.mx.z = fmaxf(a.mx.z, b.mx.z);
            s[threadIdx.x] = a;
        }
        __syncthreads();
    }
    if (threadIdx.x == 0) partial[blockIdx.x] = s[0];
}

// Morton codes (simple_knn.cu:55-71) after folding the partial bounds
__global__ __launch_bounds__(BOUNDS_THREADS) void knn_morton_kernel(int P, const float* pts, const Bounds* partial,
                                                                    int npartial, uint32_t* codes, uint32_t* idx)
{
    __shared__ Bounds s_b;
    if (threadIdx.x == 0) {
        Bounds a = partial[0];
        for (int k = 1; k < npartial; ++k) {
            const Bounds b = partial[k];
            a.mn.x = fminf(a.mn.x, b.mn.x), a.mn.y = fminf(a.mn.y, b.mn.y), a.mn.z = fminf(a.mn.z, b.mn.z);
            a.mx.x = fmaxf(a.mx.x, b.mx.x), a.mx.y = fmaxf(a.mx.y, b.mx.y), a.mx.z = fmaxf(a.mx.z, b.mx.z);
        }
        s_b = a;
    }
    __syncthreads();
    const int i = blockIdx.x * BOUNDS_THREADS + threadIdx.x;
    if (i >= P) return;
    const Bounds b = s_b;
    const float x = pts[3 * i], y = pts[3 * i + 1], z = pts[3 * i + 2];
    // float -> uint32 conversion of ((c - min) / (max - min)) * 1023, as the reference; a degenerate axis (NaN)
    // converts to 0 on gfx950 as on CUDA
    auto q = [](float c, float lo, float hi) {
        const float t = ((c - lo) / (hi - lo)) * (float)((1 << 10) - 1);
        return t == t ? (uint32_t)t : 0u;
    };
    codes[i] = prep_morton(q(x, b.mn.x, b.mx.x)) | (prep_morton(q(y, b.mn.y, b.mx.y)) << 1) |
               (prep_morton(q(z, b.mn.z, b.mx.z)) << 2);
    idx[i] = (uint32_t)i;
}

// sorted point copy (float4) and the bounds of every 64-point box; superbox bounds from their boxes
__global__ __launch_bounds__(KNN_BOX) void knn_boxes_kernel(int P, const float* pts, const uint32_t* order,
                                                            float4* spts, Bounds* boxes)
{
    const int i = blockIdx.x * KNN_BOX + threadIdx.x;
    float4 p = make_float4(FLT_MAX, FLT_MAX, FLT_MAX, 0.f);
    float4 mn = p, mx = make_float4(-FLT_MAX, -FLT_MAX, -FLT_MAX, 0.f);
    if (i < P) {
        const uint32_t g = order[i];
        p = make_float4(pts[3 * g], pts[3 * g + 1], pts[3 * g + 2], 0.f);
        spts[i] = p;
        mn = p, mx = p;
    }
    for (int o = 32; o > 0; o >>= 1) {
        mn.x = fminf(mn.x, __shfl_xor(mn.x, o, 64)), mn.y = fminf(mn.y, __shfl_xor(mn.y, o, 64));
        mn.z = fminf(mn.z, __shfl_xor(mn.z, o, 64));
        mx.x = fmaxf(mx.x, __shfl_xor(mx.x, o, 64)), mx.y = fmaxf(mx.y, __shfl_xor(mx.y, o, 64));
        mx.z = fmaxf(mx.z, __shfl_xor(mx.z, o, 64));
    }
    if (threadIdx.x == 0) boxes[blockIdx.x] = {mn, mx};
}

__global__ __launch_bounds__(KNN_BOX) void knn_superboxes_kernel(int nbox, const Bounds* boxes, Bounds* supers)
{
    const int b = blockIdx.x * KNN_SUPER + threadIdx.x;
    float4 mn = make_float4(FLT_MAX, FLT_MAX, FLT_MAX, 0.f), mx = make_float4(-FLT_MAX, -FLT_MAX, -FLT_MAX, 0.f);
    if (b < nbox) mn = boxes[b].mn, mx = boxes[b].mx;
    for (int o = 32; o > 0; o >>= 1) {
        mn.x = fminf(mn.x, __shfl_xor(mn.x, o, 64)), mn.y = fminf(mn.y, __shfl_xor(mn.y, o, 64));
        mn.z = fminf(mn.z, __shfl_xor(mn.z, o, 64));
        mx.x = fmaxf(mx.x, __shfl_xor(mx.x, o, 64)), mx.y = fmaxf(mx.y, __shfl_xor(mx.y, o, 64));
        mx.z = fmaxf(mx.z, __shfl_xor(mx.z, o, 64));
    }
    if (threadIdx.x == 0) supers[blockIdx.x] = {mn, mx};
}

// one wave per box of 64 sorted queries (simple_knn.cu:145-183 restructured; see the file header)
__global__ __launch_bounds__(KNN_BOX) void knn_query_kernel(int P, const float4* spts, const uint32_t* order,
                                                            const Bounds* boxes, const Bounds* supers, int nbox,
                                                            int nsuper, float* dists)
{
    __shared__ float4 s_pts[KNN_BOX];
    const int i = blockIdx.x * KNN_BOX + threadIdx.x;
    const bool live = i < P;
    float px = FLT_MAX, py = FLT_MAX, pz = FLT_MAX;
    if (live) {
        const float4 p = spts[i];
        px = p.x, py = p.y, pz = p.z;
    }
    // rejection radius from the +-3 sorted neighbours
    float b0 = FLT_MAX, b1 = FLT_MAX, b2 = FLT_MAX;
    if (live) {
        for (int j = max(0, i - 3); j <= min(P - 1, i + 3); ++j) {
            if (j == i) continue;
            const float4 c = spts[j];
            update_best(sqdist(px, py, pz, c.x, c.y, c.z), b0, b1, b2);
        }
    }
    const float reject = b2;
    b0 = b1 = b2 = FLT_MAX;
    for (int sb = 0; sb < nsuper; ++sb) {
        const Bounds S = supers[sb];  // wave-uniform index: scalar loads
        const float ds = box_dist(S, px, py, pz);
        if (!__any(live && !(ds > reject || ds > b2))) continue;
        const int bend = min(nbox, (sb + 1) * KNN_SUPER);
        for (int b = sb * KNN_SUPER; b < bend; ++b) {
            const Bounds B = boxes[b];
            const float db = box_dist(B, px, py, pz);
            const bool need = live && !(db > reject || db > b2);
            if (!__any(need)) continue;
            const int base = b * KNN_BOX;
            const int n = min(KNN_BOX, P - base);
            wave_sync();
            if ((int)threadIdx.x < n) s_pts[threadIdx.x] = spts[base + threadIdx.x];
            wave_sync();
            if (need) {
                for (int j = 0; j < n; ++j) {
                    if (base + j == i) continue;
                    const float4 c = s_pts[j];
                    update_best(sqdist(px, py, pz, c.x, c.y, c.z), b0, b1, b2);
                }
            }
        }
    }
    if (live) dists[order[i]] = (b0 + b1 + b2) / 3.0f;
}

size_t knn_scratch_bytes(int P)
{
    const size_t n = (size_t)std::max(P, 0);
    const size_t nbox = div_up(n, KNN_BOX), nsuper = div_up(nbox, KNN_SUPER);
    Carver c(nullptr);
    c.take<uint32_t>(n), c.take<uint32_t>(n), c.take<uint32_t>(n), c.take<uint32_t>(n);
    c.take<uint32_t>(radix_scratch_words(n, 4));
    c.take<uint32_t>(radix_partials_words(n));
    c.take<float4>(n);
    c.take<Bounds>(nbox), c.take<Bounds>(nsuper), c.take<Bounds>(BOUNDS_BLOCKS);
    return c.size();
}

void launch_knn(int P, const float* pts, float* dists, char* scratch, hipStream_t s)
{
    if (P <= 0) return;
    const size_t n = (size_t)P;
    const uint32_t nbox = div_up(n, KNN_BOX), nsuper = div_up(nbox, KNN_SUPER);
    Carver c(scratch);
    uint32_t *ka = c.take<uint32_t>(n), *kb = c.take<uint32_t>(n), *va = c.take<uint32_t>(n),
             *vb = c.take<uint32_t>(n);
    uint32_t* hist = c.take<uint32_t>(radix_scratch_words(n, 4));
    uint32_t* partials = c.take<uint32_t>(radix_partials_words(n));
    float4* spts = c.take<float4>(n);
    Bounds* boxes = c.take<Bounds>(nbox);
    Bounds* supers = c.take<Bounds>(nsuper);
    Bounds* part = c.take<Bounds>(BOUNDS_BLOCKS);
    const int nb = (int)std::min<uint32_t>(BOUNDS_BLOCKS, div_up(n, BOUNDS_THREADS));
    knn_bounds_kernel<<<nb, BOUNDS_THREADS, 0, s>>>(P, pts, part);
    knn_morton_kernel<<<div_up(n, BOUNDS_THREADS), BOUNDS_THREADS, 0, s>>>(P, pts, part, nb, ka, va);
    const int which = radix_sort_pairs(ka, kb, va, vb, hist, partials, n, nullptr, nullptr, 0, 4, s);
    const uint32_t* order = which ? vb : va;
    knn_boxes_kernel<<<nbox, KNN_BOX, 0, s>>>(P, pts, order, spts, boxes);
    knn_superboxes_kernel<<<nsuper, KNN_BOX, 0, s>>>((int)nbox, boxes, supers);
    knn_query_kernel<<<nbox, KNN_BOX, 0, s>>>(P, spts, order, boxes, supers, (int)nbox, (int)nsuper, dists);
}

}  // namespace omr
