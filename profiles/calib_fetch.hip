// calib_fetch.hip — calibrates rocprofv3 FETCH_SIZE / WRITE_SIZE on gfx950 for the access patterns the render
// kernels use (MI355X_MICROARCH.md § HBM: the x2 FETCH correction holds for 16-B/lane streaming reads only; "other
// access widths are uncalibrated: calibrate on a known byte count in your own access pattern").
//
// Every kernel moves a known number of bytes; profiles/calib_fetch.sh runs this program under two --pmc passes
// (FETCH_SIZE, WRITE_SIZE) and profiles/calib_summarize.py prints counter bytes / known bytes per pattern.
// The tables are 2 GiB (well past the 256 MiB Infinity Cache), indices are a fixed-seed hash, so gathers miss.
//
//   stream16   16-B/lane contiguous reads                          known = n * 16
//   gather64   one random 64-B aligned record per lane (4 x 16 B)   known = n * 64   (render record gather)
//   gather4    one random 4-B word per lane                         known = n * 4    (row_first[gid] gather)
//   row36      9 lanes of a wave write one random 36-B row          known = rows * 36 (render_bwd gradient rows)
//   byte1      one random byte per lane                             known = n        (row_valid marks)
//   wstream16  16-B/lane contiguous writes                          known = n * 16
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>

#define CK(x)                                                                                     \
    do {                                                                                          \
        hipError_t e_ = (x);                                                                      \
        if (e_ != hipSuccess) {                                                                   \
            std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));                          \
            std::exit(1);                                                                         \
        }                                                                                         \
    } while (0)

__device__ __forceinline__ uint64_t mix(uint64_t x)
{
    x += 0x9E3779B97F4A7C15ull;
    x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
    x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
    return x ^ (x >> 31);
}

__global__ void stream16(const float4* __restrict__ in, size_t n, float* out)
{
    float acc = 0.f;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
        const float4 v = in[i];
        acc += v.x + v.y + v.z + v.w;
    }
    if (acc == 1234.5f) out[0] = acc;  // keeps the loads; never true on the zeroed table
}

__global__ void gather64(const float4* __restrict__ table, size_t nrec, size_t n, float* out)
{
    const size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
    if (i >= n) return;
    const size_t r = mix(i) % nrec;
    const float4* p = table + r * 4;
    const float4 a = p[0], b = p[1], c = p[2], d = p[3];
    const float acc = a.x + b.y + c.z + d.w + a.w + b.x + c.y + d.z;
    if (acc == 1234.5f) out[0] = acc;
}

__global__ void gather4(const uint32_t* __restrict__ table, size_t nw, size_t n, float* out)
{
    const size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
    if (i >= n) return;
    const uint32_t v = table[mix(i + 77) % nw];
    if (v == 12345u) out[0] = 1.f;
}

__global__ void row36(float* __restrict__ rows, size_t nrows, size_t nwrite)
{
    // one row per wave, as render_bwd stores it: lanes 0, 8, .., 56 write values 0..7, lane 1 value 8
    const size_t w = (blockIdx.x * (size_t)blockDim.x + threadIdx.x) >> 6;
    const uint32_t lane = threadIdx.x & 63;
    if (w >= nwrite) return;
    float* row = rows + (mix(w + 999) % nrows) * 9;
    const bool lead = (lane & 7) == 0;
    if (lead || lane == 1) row[lead ? (lane >> 3) : 8u] = (float)lane;
}

__global__ void byte1(uint8_t* __restrict__ bytes, size_t nb, size_t n)
{
    const size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
    if (i >= n) return;
    bytes[mix(i + 4242) % nb] = 1;
}

__global__ void wstream16(float4* __restrict__ out, size_t n)
{
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
        out[i] = make_float4(1.f, 2.f, 3.f, 4.f);
}

int main()
{
    const size_t table_bytes = 2ull << 30;
    void *table, *wtable;
    float* sink;
    CK(hipMalloc(&table, table_bytes));
    CK(hipMalloc(&wtable, table_bytes));
    CK(hipMalloc(&sink, 256));
    CK(hipMemset(table, 0, table_bytes));
    CK(hipMemset(wtable, 0, table_bytes));
    CK(hipDeviceSynchronize());
    const size_t n_stream = 256ull << 20 >> 4;  // 256 MiB of 16-B reads
    const size_t n_g = 4ull << 20;              // 4 M gathers / writes
    const size_t nrec = table_bytes / 64, nw = table_bytes / 4, nrows = table_bytes / 36;
    for (int rep = 0; rep < 3; ++rep) {
        stream16<<<4096, 256>>>(static_cast<const float4*>(table), n_stream, sink);
        gather64<<<(unsigned)(n_g / 256), 256>>>(static_cast<const float4*>(table), nrec, n_g, sink);
        gather4<<<(unsigned)(n_g / 256), 256>>>(static_cast<const uint32_t*>(table), nw, n_g, sink);
        row36<<<(unsigned)(n_g * 64 / 256), 256>>>(static_cast<float*>(wtable), nrows, n_g);
        byte1<<<(unsigned)(n_g / 256), 256>>>(static_cast<uint8_t*>(wtable), table_bytes, n_g);
        wstream16<<<4096, 256>>>(static_cast<float4*>(wtable), n_stream);
    }
    CK(hipDeviceSynchronize());
    std::printf("{\"stream16\": %zu, \"gather64\": %zu, \"gather4\": %zu, \"row36\": %zu, \"byte1\": %zu, "
                "\"wstream16\": %zu}\n",
                n_stream * 16, n_g * 64, n_g * 4, n_g * 36, n_g, n_stream * 16);
    return 0;
}
