// write_bw.hip — what HBM write rate a store-only kernel reaches on this box, to price gaussian_bwd's culled rows
// (config E pinhole: 88 % of 5 M Gaussians culled, every gradient output still written once).
//   hipcc --offload-arch=gfx950 -O3 -o omnigs-fork_amd/lib/test/write_bw profiles/write_bw.hip
//   write_bw [GiB]  ->  one line per pattern: GB/s over the median of 20 launches
// Patterns: float4 grid-stride (1 KiB contiguous per wave instruction); dword stores at stride 12 B (three
// instructions per 768-B span, the AoS [P][3] outputs); the 192-B rows staged through LDS as 12 x 1 KiB spans
// (wave_rows_store). hipMemsetAsync for comparison.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CHECK(x)                                                                      \
    do {                                                                              \
        hipError_t e_ = (x);                                                          \
        if (e_ != hipSuccess) {                                                       \
            std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
            std::exit(1);                                                             \
        }                                                                             \
    } while (0)

__global__ __launch_bounds__(256) void store_f4(float4* p, size_t n)
{
    const size_t stride = (size_t)gridDim.x * blockDim.x;
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) p[i] = make_float4(0.f, 0.f, 0.f, 0.f);
}

// thread t of the grid owns element t of a [n][3] float array: three dword stores 12 B apart per lane
__global__ __launch_bounds__(256) void store_aos3(float* p, size_t n)
{
    const size_t stride = (size_t)gridDim.x * blockDim.x;
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
        p[3 * i] = 0.f;
        p[3 * i + 1] = 0.f;
        p[3 * i + 2] = 0.f;
    }
}

// one wave per 64 rows of 12 float4: each lane writes its row into LDS (odd stride 13), then the wave stores the
// 12-KiB span contiguously (instruction q, lane l -> float4 q * 64 + l)
__global__ __launch_bounds__(256) void store_rows_lds(float4* p, size_t rows)
{
    __shared__ float4 s[4][64 * 13];
    const uint32_t lane = threadIdx.x & 63u, wv = threadIdx.x >> 6;
    const size_t waves = (size_t)gridDim.x * 4;
    for (size_t w = (size_t)blockIdx.x * 4 + wv; w * 64 < rows; w += waves) {
        float4* img = s[wv];
#pragma unroll
        for (int q = 0; q < 12; ++q) img[lane * 13 + q] = make_float4(0.f, 0.f, 0.f, (float)q);
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        float4* dst = p + w * 64 * 12;
        const size_t left = rows - w * 64;
#pragma unroll
        for (int q = 0; q < 12; ++q) {
            const uint32_t k = (uint32_t)q * 64u + lane, r = k / 12u, c = k - r * 12u;
            if (r < left) dst[k] = img[r * 13 + c];
        }
        __builtin_amdgcn_wave_barrier();
    }
}

int main(int argc, char** argv)
{
    const double gib = argc > 1 ? std::atof(argv[1]) : 1.5;
    const size_t bytes = (size_t)(gib * (1ull << 30)) / 768 * 768;
    void* buf;
    CHECK(hipMalloc(&buf, bytes));
    hipEvent_t e0, e1;
    CHECK(hipEventCreate(&e0));
    CHECK(hipEventCreate(&e1));
    int cus = 0;
    CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    auto run = [&](const char* name, auto launch) {
        std::vector<float> ms;
        for (int it = 0; it < 23; ++it) {
            CHECK(hipEventRecord(e0, 0));
            launch();
            CHECK(hipEventRecord(e1, 0));
            CHECK(hipEventSynchronize(e1));
            float t;
            CHECK(hipEventElapsedTime(&t, e0, e1));
            if (it >= 3) ms.push_back(t);
        }
        std::sort(ms.begin(), ms.end());
        const float med = ms[ms.size() / 2];
        std::printf("%-28s %8.3f ms  %7.1f GB/s\n", name, med, bytes / (med * 1e-3) / 1e9);
    };
    const size_t n4 = bytes / 16, n3 = bytes / 12, nrows = bytes / 192;
    for (int g : {cus * 8, cus * 32, (int)std::min<size_t>((n4 + 255) / 256, 1u << 20)}) {
        char name[64];
        std::snprintf(name, sizeof name, "float4 grid=%d", g);
        run(name, [&] { store_f4<<<g, 256>>>((float4*)buf, n4); });
    }
    run("aos3 dword (full grid)", [&] { store_aos3<<<(unsigned)((n3 + 255) / 256), 256>>>((float*)buf, n3); });
    run("rows via LDS (full grid)", [&] { store_rows_lds<<<(unsigned)((nrows + 255) / 256), 256>>>((float4*)buf, nrows); });
    run("rows via LDS grid=8/CU", [&] { store_rows_lds<<<cus * 8, 256>>>((float4*)buf, nrows); });
    run("hipMemsetAsync", [&] { CHECK(hipMemsetAsync(buf, 0, bytes, 0)); });
    CHECK(hipFree(buf));
    return 0;
}
