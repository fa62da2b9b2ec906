// capi.hip — orchestration of the gfx950 rasterizer behind the C ABI of include/omnigs_raster.h.
//
// Forward  (reference: LonlatRasterizer::forward / Rasterizer::forward, rasterizer_impl.cu:540-697 / :250-433):
//   preprocess -> depth sort of Gaussians -> scan of tiles_touched in depth order -> [one host sync for
//   num_rendered] -> emit instances -> tile sort -> tile ranges -> render.
// Backward (reference: LonlatRasterizer::backward / Rasterizer::backward, rasterizer_impl.cu:701-795 / :437-535):
//   render backward (per-instance gradient rows) -> fused per-Gaussian backward.
// Everything is enqueued on the caller's stream; no allocation happens outside the three callbacks.
#include <algorithm>
#include <atomic>
#include <chrono>
#include <deque>
#include <mutex>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

#include "../../include/omnigs_raster.h"
#include "kernels.h"
#include "tile_wave.h"
#include "wave_ops.h"

namespace omr {

namespace {

// one wave: in [64][9] -> out[9] through wave_sum9_rows (the row sums' long-Gaussian reduction)
__global__ __launch_bounds__(64) void debug_wave_sum9_kernel(const float* in, float* out)
{
    const uint32_t lane = threadIdx.x;
    float v[8];
#pragma unroll
    for (int c = 0; c < 8; ++c) v[c] = in[lane * 9 + c];
    float t8;
    const float tv = wave_sum9_rows(v, in[lane * 9 + 8], lane, &t8);
    if ((lane & 7) == 0) out[lane >> 3] = tv;
    if (lane == 1) out[8] = t8;
}

// the same through wave_sum9_lds (the render backward's unpaired reduction)
__global__ __launch_bounds__(64) void debug_wave_sum9_lds_kernel(const float* in, float* out)
{
    __shared__ __attribute__((aligned(16))) float s_red[8 * WS_LDS_STRIDE];
    const uint32_t lane = threadIdx.x;
    float v[8];
#pragma unroll
    for (int c = 0; c < 8; ++c) v[c] = in[lane * 9 + c];
    float t8;
    const float tv = wave_sum9_lds(v, in[lane * 9 + 8], lane, s_red, &t8);
    if ((lane & 7) == 0) out[lane >> 3] = tv;
    if (lane == 1) out[8] = t8;
}

// two instances' rows through wave_sum9x2_stored (the render backward's paired reduction): in is
// [2][64][9], out [2][9]
__global__ __launch_bounds__(64) void debug_wave_sum9x2_kernel(const float* in, float* out)
{
    __shared__ __attribute__((aligned(16))) float s_red[16 * WS_LDS_STRIDE];
    const uint32_t lane = threadIdx.x;
#pragma unroll
    for (int k = 0; k < 16; ++k) s_red[k * WS_LDS_STRIDE + lane] = in[(k >> 3) * 576 + lane * 9 + (k & 7)];
    float t8;
    const float tv = wave_sum9x2_stored(in[lane * 9 + 8], in[576 + lane * 9 + 8], lane, s_red, &t8);
    const uint32_t k = lane >> 2;
    if ((lane & 3) == 0) out[(k >> 3) * 9 + (k & 7)] = tv;
    if ((lane & 31) == 1) out[(lane >> 5) * 9 + 8] = t8;
}

// the DPP wave scans of raster_common.h (every block scan of the sorts and the binning): in [2][64] u32, out [3][64] =
// inclusive sum of in[0], inclusive max of in[1], the wave max of in[1] on every lane (tile_wave.h)
__global__ __launch_bounds__(64) void debug_wave_scans_kernel(const uint32_t* in, uint32_t* out)
{
    const uint32_t lane = threadIdx.x;
    out[lane] = wave_incl_sum_u32(in[lane]);
    out[64 + lane] = wave_incl_max_u32(in[64 + lane]);
    out[128 + lane] = wave_max_u32(in[64 + lane]);
}

__global__ __launch_bounds__(256) void debug_point_ids_kernel(const uint32_t* list, size_t n, uint32_t* out)
{
    const size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;
    if (i < n) out[i] = list[i] & PL_GID_MASK;
}

thread_local std::string g_last_error;
// omr_backward_colors_event: recorded by this thread's next backward once dL_dcolor is final, then cleared
thread_local hipEvent_t t_colors_event = nullptr;
// omr_backward_chunk_events: the next backward on this thread runs gaussian_bwd over that many Gaussian ranges and
// records one event after each (omr_backward_chunk_begin gives the ranges), then forgets them
thread_local std::vector<hipEvent_t> t_chunk_events;

int fail(int code, const std::string& msg)
{
    g_last_error = msg;
    return code;
}

int hip_check(const char* where)
{
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) return fail(OMR_ERR_HIP, std::string(where) + ": " + hipGetErrorString(e));
    return OMR_OK;
}

#define OMR_HIP(call)                                                                            \
    do {                                                                                         \
        const hipError_t e_ = (call);                                                            \
        if (e_ != hipSuccess) return fail(OMR_ERR_HIP, std::string(#call) + ": " + hipGetErrorString(e_)); \
    } while (0)

// ---- stage profiler: hipEvent pairs on the launch stream, resolved lazily by omr_profile_read -------------
enum Stage { ST_PREPROCESS, ST_DEPTH_SORT, ST_SCAN, ST_EMIT, ST_TILE_SORT, ST_RANGES, ST_RENDER_FWD, ST_RENDER_BWD,
             ST_GAUSS_BWD, ST_ROW_SUMS, ST_COUNT };
const char* kStageNames[ST_COUNT] = {"preprocess", "depth_sort", "scan", "emit", "tile_sort", "tile_ranges",
                                     "render_forward", "render_backward", "gaussian_backward", "row_sums"};

// Diagnostic (bench.py, tests): one process-wide profiler, guarded by a mutex; its events belong to the device that
// was current when they were created, so profile one device per process.
struct Profiler {
    std::mutex mu;
    bool on = false;
    uint32_t mask = ~0u;
    struct Rec {
        int stage;
        hipEvent_t a, b;
    };
    std::vector<Rec> pending;
    std::vector<hipEvent_t> pool;
    double total_ms[ST_COUNT] = {};
    uint64_t count[ST_COUNT] = {};
    hipEvent_t get()  // caller holds mu
    {
        if (!pool.empty()) {
            hipEvent_t e = pool.back();
            pool.pop_back();
            return e;
        }
        // timing only: no system-scope fence (an L2 writeback + invalidate, about 5 us of GPU idle per event)
        hipEvent_t e = nullptr;
        if (hipEventCreateWithFlags(&e, hipEventDisableSystemFence) != hipSuccess)
            return nullptr;
        return e;
    }
};
Profiler g_prof;

// A stage of several launches is bracketed by two event records. Each is a marker packet whose system-scope release
// writes back the L2 (about 6 us of GPU idle at config C, profiles/gaps.py), so a single-kernel stage (single = true)
// instead hands its pair to the launch (start(), stop()), which attaches it to the dispatch packet
// (hipExtLaunchKernelGGL): the timed pass that measures the roofline kernel then costs no idle time.
struct StageScope {
    int stage;
    hipStream_t s;
    bool single;
    hipEvent_t a = nullptr, b = nullptr;
    StageScope(int st, hipStream_t stream, bool single_kernel = false)
        : stage(st), s(stream), single(single_kernel)
    {
        if (g_prof.on && (g_prof.mask >> st) & 1u) {
            std::lock_guard<std::mutex> lk(g_prof.mu);
            a = g_prof.get();
            if (a && single) {
                b = g_prof.get();
                if (!b) a = nullptr;
            } else if (a) {
                (void)hipEventRecord(a, s);
            }
        }
    }
    hipEvent_t start() const { return single ? a : nullptr; }
    hipEvent_t stop() const { return single ? b : nullptr; }
    ~StageScope()
    {
        if (a) {
            std::lock_guard<std::mutex> lk(g_prof.mu);
            if (!single) {
                b = g_prof.get();
                if (b) (void)hipEventRecord(b, s);
            }
            if (b) g_prof.pending.push_back({stage, a, b});
        }
    }
};

// Host-visible words the forward and backward read back, per (thread, device): a forward may run on any device's
// stream, and an event can only be recorded on a stream of the device it was created on.
//   words[0..3] <- counters[0..3] after the forward's scan (num_rendered, prefiltered flag, huge count, error word)
//   words[4]    <- counters[3] at the start of the backward (look-back errors of the forward's back half)
//   words[6], words[7]: the sequence numbers written after them (HostRead)
// The words the host reads back (num_rendered etc.) are written by the GPU straight into pinned fine-grained memory
// with system-scope stores by the first wave of a kernel that runs anyway, followed by a sequence number the host
// spins on (kernels.h: HostWords): no blit kernel and no event. Either of those costs a dispatch and ends in a
// system-scope release that writes back the L2 — about 5 us of GPU idle each at config C (profiles/gaps.py).
// (A hipMemcpyAsync + event record + event wait instead cost about 14 us of GPU idle per step at config C.)
// one host read-back: data words + the sequence word the GPU writes after them
struct HostRead {
    uint32_t* host;       // data, host address
    uint32_t* dev;        // data, device address
    uint32_t* seq_host;   // sequence word
    uint32_t* seq_dev;
    uint32_t seq = 0;     // last value requested
};

// Requests src_dev[0..n) into r's words. Returns what the next launch that carries host words (emit_index,
// backward_schedule) must write, or dst == NULL when the request is already queued (own kernel).
HostWords read_to_host(HostRead& r, const uint32_t* src_dev, int n, hipStream_t s, bool own_kernel, hipError_t* err)
{
    HostWords h;
    *err = hipSuccess;
    h.dst = r.dev;
    h.src = src_dev;
    h.n = n;
    h.seq_dst = r.seq_dev;
    h.seq = ++r.seq;
    if (own_kernel) {
        launch_host_words(h, s);
        *err = hipGetLastError();
        h.dst = nullptr;
    }
    return h;
}

// waits for the words of the last read_to_host. The stream is queried only after 50 ms of polling (a stream
// query enqueues a marker, which costs the GPU the same idle time as an event): it fails the wait if the stream
// reports an error or has drained without the words.
hipError_t wait_host_read(const HostRead& r, hipStream_t s)
{
    const auto t0 = std::chrono::steady_clock::now();
    uint32_t polls = 0;
    while (__atomic_load_n(r.seq_host, __ATOMIC_ACQUIRE) != r.seq) {
        if ((++polls & 1023u) == 0 && std::chrono::steady_clock::now() - t0 > std::chrono::milliseconds(50)) {
            const hipError_t q = hipStreamQuery(s);
            if (q != hipSuccess && q != hipErrorNotReady) return q;
            if (q == hipSuccess && __atomic_load_n(r.seq_host, __ATOMIC_ACQUIRE) != r.seq) return hipErrorUnknown;
            std::this_thread::sleep_for(std::chrono::microseconds(100));
        }
    }
    return hipSuccess;
}

struct HostSlots {
    int device = -1;
    uint32_t* words = nullptr;
    uint32_t* words_dev = nullptr;  // the same words as the device addresses them
    HostRead fwd, bwd;              // words[0..3] | words[4], sequence words[6] | words[7]
};

int stream_device(hipStream_t s)
{
    int dev = 0;
    if (s) {
        hipDevice_t d;
        if (hipStreamGetDevice(s, &d) == hipSuccess) return (int)d;
    }
    (void)hipGetDevice(&dev);
    return dev;
}

HostSlots* host_slots(hipStream_t s)
{
    thread_local std::deque<HostSlots> slots;  // deque: pointers stay valid as devices are added
    const int dev = stream_device(s);
    for (auto& h : slots)
        if (h.device == dev) return &h;
    int cur = dev;
    (void)hipGetDevice(&cur);
    if (cur != dev && hipSetDevice(dev) != hipSuccess) return nullptr;
    HostSlots h;
    h.device = dev;
    const bool ok = hipHostMalloc(reinterpret_cast<void**>(&h.words), 8 * sizeof(uint32_t),
                                  hipHostMallocPortable | hipHostMallocCoherent | hipHostMallocMapped) == hipSuccess &&
                    hipHostGetDevicePointer(reinterpret_cast<void**>(&h.words_dev), h.words, 0) == hipSuccess;
    if (ok) {
        std::memset(h.words, 0, 8 * sizeof(uint32_t));
        h.fwd.host = h.words;
        h.fwd.dev = h.words_dev;
        h.fwd.seq_host = h.words + 6;
        h.fwd.seq_dev = h.words_dev + 6;
        h.bwd.host = h.words + 4;
        h.bwd.dev = h.words_dev + 4;
        h.bwd.seq_host = h.words + 7;
        h.bwd.seq_dev = h.words_dev + 7;
    }
    if (cur != dev) (void)hipSetDevice(cur);
    if (!ok) return nullptr;
    slots.push_back(h);
    return &slots.back();
}

// process-wide counters of what the host side of the rasterizer did (omr_runtime_stats): evidence for host stalls
enum RtStat { RS_FORWARDS, RS_BACKWARDS, RS_FIRST_CALL_SYNCS, RS_BACK_HALF_RERUNS, RS_COUNT_WAIT_NS, RS_BWD_WAIT_NS,
              RS_ALLOC_CALLS, RS_ALLOC_BYTES, RS_LOOKBACK_ERRORS, RS_COUNT };
const char* kRtStatNames[RS_COUNT] = {"forwards", "backwards", "first_call_syncs", "back_half_reruns", "count_wait_ns",
                                      "backward_wait_ns", "alloc_calls", "alloc_bytes", "lookback_errors"};
std::atomic<uint64_t> g_rt[RS_COUNT];
void rt_add(int k, uint64_t v) { g_rt[k].fetch_add(v, std::memory_order_relaxed); }

// host wait on an event, timed into a runtime counter
hipError_t timed_wait(const HostRead& hr, hipStream_t s, int stat)
{
    const auto t0 = std::chrono::steady_clock::now();
    const hipError_t r = wait_host_read(hr, s);
    rt_add(stat, (uint64_t)std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::steady_clock::now() - t0).count());
    return r;
}

void* alloc_counted(omr_alloc_fn fn, void* ctx, size_t bytes)
{
    rt_add(RS_ALLOC_CALLS, 1);
    rt_add(RS_ALLOC_BYTES, bytes);
    return fn(ctx, bytes);
}

// per-thread capacity hint for the binning buffer, by view shape (L depends mostly on the resolution and camera)
size_t& capacity_hint(int W, int H, int camera_type)
{
    struct Entry {
        int W, H, cam;
        size_t hint;
    };
    thread_local std::vector<Entry> table;
    for (auto& e : table)
        if (e.W == W && e.H == H && e.cam == camera_type) return e.hint;
    if (table.size() >= 16) table.erase(table.begin());
    table.push_back({W, H, camera_type, 0});
    return table.back().hint;
}

}  // namespace

size_t GeomState::carve(char* base, size_t P, GeomState* s, bool rows, bool jac)
{
    Carver c(base);
    GeomState g;
    g.splat = c.take<float4>(P * SPLAT_F4);
    g.clamped = c.take<uint8_t>(P);
    g.tiles_touched = c.take<uint32_t>(P);
    g.key_a = c.take<uint32_t>(P);
    g.key_b = c.take<uint32_t>(P);
    g.val_a = c.take<uint32_t>(P);
    g.val_b = c.take<uint32_t>(P);
    g.hist = c.take<uint32_t>(depth_sort_scratch_words(P));  // also fits the plain sort (OMR_DEPTH_SORT=bytes)
    g.scan_partials = c.take<uint32_t>(depth_sort_partials_words(P));
    g.scan2_status = c.take<uint32_t>(scan2_status_words(P));
    g.offsets = c.take<uint32_t>(P);
    g.counters = c.take<uint32_t>(8);
    g.row_first = c.take<uint32_t>(P);
    g.row_sums = c.take<float>(P * GRAD_ROW);
    g.conic_op = c.take<float4>(P);
    g.huge_list = c.take<uint32_t>(P);
    g.internal_radii = c.take<int>(P);
    g.order = c.take<uint32_t>(P);
    // the optional tail: the row binning's arrays (bin.hip; preprocess and the forward scans write them only when
    // present), then sh_jac (preprocess writes it exactly when sh_jac_stored holds, which is when the forward carves it)
    if (rows) {
        g.rect = c.take<uint2>(P);
        g.drect = c.take<uint2>(P);
        g.row_offsets = c.take<uint32_t>(P);
        g.desc_r = c.take<uint2>(P / 2 + 2);  // M <= BIN_MAX_GRID P slots: at most P / 2 + 1 chunks
        g.bin_rec = c.take<float4>(2 * P);
    } else {
        g.rect = g.drect = g.desc_r = nullptr;
        g.row_offsets = nullptr;
        g.bin_rec = nullptr;
    }
    g.sh_jac = jac ? c.take<float>(9 * P) : nullptr;
    if (s) *s = g;
    return c.size();
}

static int* geom_internal_radii(char* base, size_t P)
{
    GeomState g;
    GeomState::carve(base, P, &g);
    return g.internal_radii;
}

size_t ImageState::carve(char* base, size_t N, size_t T, ImageState* s)
{
    Carver c(base);
    ImageState im;
    im.final_T = c.take<float>(N);
    im.n_contrib = c.take<uint32_t>(N);
    im.ranges = c.take<uint2>(T);
    im.tile_order = c.take<uint32_t>(T);
    im.tile_cost = c.take<uint32_t>(T);
    im.max_contrib = c.take<uint32_t>(T * FWD_GROUPS);
    im.final_C = c.take<float>(3 * N);
    if (s) *s = im;
    return c.size();
}

// The binning: the row binning (bin.hip) on views of more than BIN_SORT_MAX_TILES tiles and at most BIN_MAX_GRID
// tiles a side; the emit + radix tile sort (sort.hip) otherwise. On the smallest views the sort path's four launches
// beat the row binning's seven (config A: 967 -> 1003 MP/s; B, 2048 tiles: 2010 vs 1978, profiles/r06r_ab_{A,B}.txt).
// omr_debug_binning_mode / OMR_BINNING=rows|sort (the start value) force either for tests and A/B runs; a forward and
// its backward must see the same mode (the binning buffer's layout follows it).
static std::atomic<int>& binning_mode()  // 0: by view, 1: rows (where the grid allows), 2: sort
{
    static std::atomic<int> mode{[] {
        const char* v = std::getenv("OMR_BINNING");
        if (v && std::strcmp(v, "rows") == 0) return 1;
        if (v && std::strcmp(v, "sort") == 0) return 2;
        return 0;
    }()};
    return mode;
}
// The depth sort: pinhole views take depth_sort (sort.hip), whose first pass sets the culled Gaussians aside so the
// other three sort the visible keys alone (config E pinhole culls 88 %: 0.206 -> 0.137 ms); lonlat views cull only
// what is too close to the camera, and there the plain 4 x 8-bit radix sort of every key is 2-4 us faster (C 0.0795
// vs 0.0812 ms, A 0.029 vs 0.033: profiles/r05e_ab_*.txt). The same permutation either way. OMR_DEPTH_SORT (read once)
// forces one for A/B runs and tests: "bytes" the plain sort, "visible" depth_sort, "count" depth_count_sort.
// Views of at most DEPTH_COUNT_SORT_MAX Gaussians take depth_count_sort (one launch instead of five chained ones).
static std::atomic<int>& depth_sort_mode()  // 0: by size and camera type, 1: plain, 2: depth_sort, 3: count
{                                           // (omr_debug_depth_sort_mode)
    static std::atomic<int> mode{[] {
        const char* v = std::getenv("OMR_DEPTH_SORT");
        if (v && std::strcmp(v, "bytes") == 0) return 1;
        if (v && std::strcmp(v, "visible") == 0) return 2;
        if (v && std::strcmp(v, "count") == 0) return 3;
        return 0;
    }()};
    return mode;
}
static int depth_sort_forced() { return depth_sort_mode().load(std::memory_order_relaxed); }
// Adam's f_dc + f_rest row walk (adam_impl): 1 on by default, 0 the gathering groups (omr_debug_adam_sh_rows;
// OMR_ADAM_SH_ROWS=0 sets the start value)
static std::atomic<int>& adam_sh_rows_mode()
{
    static std::atomic<int> mode{[] {
        const char* v = std::getenv("OMR_ADAM_SH_ROWS");
        return (v && std::strcmp(v, "0") == 0) ? 0 : 1;
    }()};
    return mode;
}
enum DepthSortKind { DS_PLAIN, DS_VISIBLE, DS_COUNT };
static DepthSortKind depth_sort_kind(int camera_type, size_t P)
{
    const int f = depth_sort_forced();
    if (f == 3 && P <= DEPTH_COUNT_SORT_FORCED_MAX) return DS_COUNT;  // forced: any size a test can afford
    if (f == 1 || f == 2) return f == 1 ? DS_PLAIN : DS_VISIBLE;
    if (f == 0 && P <= DEPTH_COUNT_SORT_MAX) return DS_COUNT;
    return camera_type != CAM_PINHOLE ? DS_PLAIN : DS_VISIBLE;
}
static bool row_binning(uint32_t gx, uint32_t gy)
{
    const int m = binning_mode().load(std::memory_order_relaxed);
    if (m == 2 || gx > BIN_MAX_GRID || gy > BIN_MAX_GRID) return false;
    return m == 1 || (size_t)gx * gy > BIN_SORT_MAX_TILES;
}

size_t BinningState::carve(char* base, size_t cap, uint32_t gx, uint32_t gy, BinningState* s)
{
    const uint32_t T = gx * gy;
    const int tile_passes = tile_sort_passes(T);
    const bool rows = row_binning(gx, gy);
    Carver c(base);
    BinningState b;
    b.inst_grad = c.take<float>(cap * GRAD_ROW);
    // room for the rest of the L-indexed region when L < cap (raster_common.h): point list, row_valid, the
    // backward's checkpoints, per-segment work and schedule
    c.take<uint8_t>(l_region_end(cap, T) - canonical_list_offset(cap));
    b.point_list = base ? reinterpret_cast<uint32_t*>(base + canonical_list_offset(cap)) : nullptr;
    b.row_valid = base ? reinterpret_cast<uint8_t*>(base + row_valid_offset(cap)) : nullptr;
    b.key_a = c.take<uint32_t>(cap);
    b.key_b = c.take<uint32_t>(cap);
    b.val_a = c.take<uint32_t>(cap);
    b.val_b = c.take<uint32_t>(rows ? 0 : cap);
    b.hist = c.take<uint32_t>(rows ? 0 : radix_scratch_words(cap, tile_passes));
    b.scan_partials = c.take<uint32_t>(rows ? 0 : radix_partials_words(cap));  // look-back words of the histogram scan
    b.block_owner = c.take<uint32_t>(rows ? 0 : emit_index_size(cap));
    b.point_keys = (tile_passes & 1) != 0 ? b.key_b : b.key_a;  // result buffer of the key ping-pong
    b.bin_hist_r = c.take<uint32_t>(rows ? 2 * (size_t)gy * bin_chunks_r(cap) : 0);
    b.bin_hist_b = c.take<uint32_t>(rows ? bin_chunks_b(cap, gy) * gx : 0);
    b.bin_desc_b = c.take<uint4>(rows ? 2 * bin_chunks_b(cap, gy) : 0);
    b.bin_words = c.take<uint32_t>(rows ? 4 : 0);
    b.bin_zero = c.take<uint32_t>(rows ? bin_zero_words(cap, gx, gy) : 0);
    if (s) *s = b;
    return c.size();
}

namespace {

struct Dims {
    int W, H;
    uint32_t gx, gy, T;
    size_t N;
};
Dims dims(int width, int height)
{
    Dims d;
    d.W = width;
    d.H = height;
    d.gx = (uint32_t)((width + BLOCK_X - 1) / BLOCK_X);
    d.gy = (uint32_t)((height + BLOCK_Y - 1) / BLOCK_Y);
    d.T = d.gx * d.gy;
    d.N = (size_t)width * height;
    return d;
}

struct ForwardIn {
    int camera_type;
    omr_alloc_fn geometry_alloc, binning_alloc, image_alloc;
    void *geometry_ctx, *binning_ctx, *image_ctx;
    int P, D, M;
    const float* background;
    int width, height;
    const float *means3D, *shs, *colors_precomp, *opacities, *scales;
    float scale_modifier;
    const float *rotations, *cov3D_precomp, *viewmatrix, *projmatrix, *cam_pos;
    float tan_fovx, tan_fovy;
    bool prefiltered;
    float* out_color;
    int* radii;
    bool render_depth;
    hipStream_t stream;
    int* num_rendered;
};

int forward_impl(const ForwardIn& in)
{
    g_last_error.clear();
    if (in.num_rendered) *in.num_rendered = 0;
    if (in.camera_type != CAM_PINHOLE && in.camera_type != CAM_LONLAT)
        return fail(OMR_ERR_CAMERA_TYPE, "[CudaRasterizer]Invalid camera_type");
    if (in.P < 0 || in.width <= 0 || in.height <= 0) return fail(OMR_ERR_INVALID_ARGUMENT, "bad P / width / height");
    if (in.P == 0) return OMR_OK;  // rasterize_points.cu:97: nothing runs, image stays zero
    if ((uint32_t)in.P > PL_GID_MASK + 1u)  // point list entries hold the index in 28 bits (raster_common.h)
        return fail(OMR_ERR_INVALID_ARGUMENT, "P above 2^28 Gaussians per view");
    if (!in.means3D || !in.opacities || !in.viewmatrix || !in.background || !in.out_color)
        return fail(OMR_ERR_INVALID_ARGUMENT, "missing required input pointer");
    if (!in.colors_precomp && (!in.shs || in.M <= 0))
        return fail(OMR_ERR_INVALID_ARGUMENT, "either shs (M > 0) or colors_precomp is required");
    if (!in.cov3D_precomp && (!in.scales || !in.rotations))
        return fail(OMR_ERR_INVALID_ARGUMENT, "either scales+rotations or cov3D_precomp is required");
    if (in.camera_type == CAM_PINHOLE && !in.projmatrix) return fail(OMR_ERR_INVALID_ARGUMENT, "pinhole needs projmatrix");
    if (in.colors_precomp == nullptr && (in.shs == nullptr || in.cam_pos == nullptr))
        return fail(OMR_ERR_INVALID_ARGUMENT, "SH colours need cam_pos");
    const Dims d = dims(in.width, in.height);
    const hipStream_t s = in.stream;
    const size_t P = (size_t)in.P;

    const bool rows_path = row_binning(d.gx, d.gy);  // bin.hip; sort.hip's emit + tile sort for larger views
    const bool jac = sh_jac_stored(in.colors_precomp, in.M, in.shs);
    char* geom_base = static_cast<char*>(
        alloc_counted(in.geometry_alloc, in.geometry_ctx, GeomState::carve(nullptr, P, nullptr, rows_path, jac)));
    if (!geom_base) return fail(OMR_ERR_ALLOCATION, "geometry allocation failed");
    GeomState g;
    GeomState::carve(geom_base, P, &g, rows_path, jac);
    char* img_base = static_cast<char*>(alloc_counted(in.image_alloc, in.image_ctx, ImageState::carve(nullptr, d.N, d.T, nullptr)));
    if (!img_base) return fail(OMR_ERR_ALLOCATION, "image allocation failed");
    ImageState im;
    ImageState::carve(img_base, d.N, d.T, &im);
    int* radii = in.radii ? in.radii : geom_internal_radii(geom_base, P);

    // counters[1] is the prefiltered-cull flag, set by preprocess itself: cleared first, and only when it can be set
    if (in.prefiltered) OMR_HIP(hipMemsetAsync(g.counters + 1, 0, sizeof(uint32_t), s));
    PreprocessArgs pa;
    pa.zero[0] = {g.counters + 2, 2};                                  // huge-list count (scan), look-back error word
    pa.zero[1] = {reinterpret_cast<uint32_t*>(im.ranges), 2 * (size_t)d.T};  // tile_ranges writes boundaries only
    pa.zero[2] = {im.tile_cost, (size_t)d.T};                          // render_forward adds into it
    const DepthSortKind dsk = depth_sort_kind(in.camera_type, P);
    pa.zero[3] = dsk == DS_PLAIN     ? radix_zero_span(g.hist, P, DEPTH_SORT_PASSES)
                 : dsk == DS_VISIBLE ? depth_sort_zero_span(g.hist, P)  // the depth sort's digit totals / tickets / words
                                     : ZeroSpan{};
    pa.zero[4] = {g.scan2_status, scan2_status_words(P)};             // the forward scans' look-back words
    pa.P = in.P; pa.D = in.D; pa.M = in.M; pa.W = in.width; pa.H = in.height; pa.gx = d.gx; pa.gy = d.gy;
    pa.means3D = in.means3D; pa.scales = in.scales; pa.scale_modifier = in.scale_modifier; pa.rotations = in.rotations;
    pa.opacities = in.opacities; pa.shs = in.shs; pa.cov3D_precomp = in.cov3D_precomp; pa.colors_precomp = in.colors_precomp;
    pa.viewmatrix = in.viewmatrix; pa.projmatrix = in.projmatrix; pa.campos = in.cam_pos;
    pa.tan_fovx = in.tan_fovx; pa.tan_fovy = in.tan_fovy;
    pa.focal_y = (float)in.height / (2.0f * in.tan_fovy);  // rasterizer_impl.cu:275-276
    pa.focal_x = (float)in.width / (2.0f * in.tan_fovx);
    pa.prefiltered = in.prefiltered ? 1 : 0;
    pa.radii = radii;
    pa.g = g;
    pa.error_flag = reinterpret_cast<int*>(g.counters + 1);
    { StageScope st_(ST_PREPROCESS, s); launch_preprocess(in.camera_type, pa, s); }

    // depth order of the Gaussians (stable: ties keep index order)
    uint32_t* const err_dev = g.counters + 3;  // every decoupled look-back of the forward reports a give-up here
    {
        StageScope st_(ST_DEPTH_SORT, s);
        if (dsk == DS_PLAIN) {  // the plain 4 x 8-bit radix sort over all P keys
            const int which = radix_sort_pairs(g.key_a, g.key_b, g.val_a, g.val_b, g.hist, g.scan_partials, P, nullptr,
                                               nullptr, 0, DEPTH_SORT_PASSES, s, true, err_dev);
            g.order = which ? g.val_b : g.val_a;
        } else if (dsk == DS_COUNT) {  // small views: by counting, one launch
            g.order = g.val_b;
            depth_count_sort(g.key_a, g.order, P, s);
        } else {
            depth_sort(g.key_a, g.key_b, g.val_a, g.val_b, g.order, g.hist, g.scan_partials, P, s, err_dev);
        }
    }
    // after the culled-aside depth sort, depth ranks from nvis on are culled Gaussians: the scans skip their words
    // (OMR_SCAN_NVIS=0 builds: every rank, for A/B runs)
#ifndef OMR_SCAN_NVIS
#define OMR_SCAN_NVIS 1
#endif
    {
        StageScope st_(ST_SCAN, s);
        const uint32_t* nvis = dsk == DS_VISIBLE && OMR_SCAN_NVIS ? depth_sort_nvis(g.hist, P) : nullptr;
        launch_forward_scans(g.tiles_touched, rows_path ? g.rect : nullptr, g.order, g.offsets, g.row_first, g.row_offsets,
                             g.drect, g.desc_r, g.huge_list, g.counters + 2, g.scan2_status, g.counters, err_dev, P, s,
                             nvis);
    }

    // num_rendered = offsets[P-1] (+ the prefiltered error flag) to pinned host memory, without waiting for it:
    // the binning buffer is sized from a capacity hint and everything after the scan reads the count on the device,
    // so the GPU never idles on this host round trip (the reference synchronises here, rasterizer_impl.cu:628).
    // The host checks the count once the rest of the forward is queued; a hint that was too small costs one
    // re-run of the back half with the exact size.
    HostSlots* hs = host_slots(s);
    if (!hs) return fail(OMR_ERR_HIP, "pinned host memory / event allocation failed");
    uint32_t* host = hs->words;
    const uint32_t* count_dev = g.counters;  // {num_rendered, -, -, error word}: raster_common.h binning_count
    // one copy: num_rendered (scan), prefiltered flag (preprocess; meaningful only when prefiltered is set), huge
    // count, look-back error word (depth sort, scan)
    hipError_t rerr;
    // carried by the back half's first kernel; on the first call for a view shape (the count is needed before the
    // back half is sized) by its own kernel
    HostWords count_words = read_to_host(hs->fwd, g.counters, 4, s, capacity_hint(in.width, in.height, in.camera_type) == 0, &rerr);
    OMR_HIP(rerr);
    rt_add(RS_FORWARDS, 1);

    const int tile_passes = tile_sort_passes(d.T);
    // tile ids below 2^16: the tile sort moves 16-bit keys (emit, both passes and the ranges read 2 B less per key)
    const bool keys16 = d.T <= 65536u;
    size_t& hint = capacity_hint(in.width, in.height, in.camera_type);
    bool known = false;
    size_t L = 0;
    auto wait_count = [&]() -> int {
        OMR_HIP(timed_wait(hs->fwd, s, RS_COUNT_WAIT_NS));
        if (int e = hip_check("preprocess/sort/scan")) return e;
        if (in.prefiltered && host[1] != 0)
            return fail(OMR_ERR_PREFILTERED, "Point is filtered although prefiltered is set. This shouldn't happen!");
        if (host[3] != 0) {
            rt_add(RS_LOOKBACK_ERRORS, 1);
            return fail(OMR_ERR_HIP, "depth sort / scan: a decoupled look-back gave up waiting for a predecessor");
        }
        L = host[0];
        known = true;
        return OMR_OK;
    };
    if (hint == 0) {  // first call for this view shape: learn L the reference's way
        rt_add(RS_FIRST_CALL_SYNCS, 1);
        if (int e = wait_count()) return e;
    }
    size_t cap = known ? L : hint;

    bool rerun = false;  // a second back half must clear what the first one wrote (preprocess zeroed it once)
    auto back_half = [&](size_t capacity) -> int {
        if (ckpt_bytes(capacity) >= 0x80000000ull)  // 32-bit buffer offsets of the checkpoints (raster_common.h)
            return fail(OMR_ERR_INVALID_ARGUMENT, "more than 2^28 Gaussian x tile instances in one view");
        char* bin_base = static_cast<char*>(
            alloc_counted(in.binning_alloc, in.binning_ctx, BinningState::carve(nullptr, capacity, d.gx, d.gy, nullptr)));
        if (!bin_base) return fail(OMR_ERR_ALLOCATION, "binning allocation failed");
        BinningState b;
        BinningState::carve(bin_base, capacity, d.gx, d.gy, &b);
        if (rerun) OMR_HIP(hipMemsetAsync(im.ranges, 0, d.T * sizeof(uint2), s));
        if (rows_path) {
            // the binning as two counting passes (bin.hip): the whole of it is timed as the tile_sort stage
            BinArgs ba;
            ba.hw = count_words; ba.P = in.P; ba.gx = d.gx; ba.gy = d.gy; ba.cap = capacity;
            ba.counters = g.counters; ba.err = err_dev; ba.order = g.order; ba.row_offsets = g.row_offsets;
            ba.splat = g.splat; ba.bin_rec = g.bin_rec;
            ba.ent_gid = b.key_a; ba.ent_w = b.key_b; ba.ent_ex = b.val_a;
            ba.hist_r = b.bin_hist_r; ba.chunks_r = bin_chunks_r(capacity); ba.desc_r = g.desc_r; ba.drect = g.drect;
            ba.hist_b = b.bin_hist_b; ba.chunks_b = bin_chunks_b(capacity, d.gy); ba.desc_b = b.bin_desc_b;
            ba.words = b.bin_words; ba.zero = b.bin_zero; ba.nzero = 0;
            ba.ranges = im.ranges; ba.binning = bin_base;
            StageScope st_(ST_TILE_SORT, s);
            launch_row_binning(ba, s);
        } else {
            { StageScope st_(ST_EMIT, s); launch_emit_instances(count_words, in.P, capacity, count_dev, g, d.gx, b.block_owner, b.key_a, keys16, b.val_a, bin_base, s); }
            {
                StageScope st_(ST_TILE_SORT, s);
                if (keys16)
                    radix_sort_pairs(reinterpret_cast<uint16_t*>(b.key_a), reinterpret_cast<uint16_t*>(b.key_b), b.val_a,
                                     b.val_b, b.hist, b.scan_partials, capacity, count_dev, bin_base, 0, tile_passes, s,
                                     false, err_dev);
                else
                    radix_sort_pairs(b.key_a, b.key_b, b.val_a, b.val_b, b.hist, b.scan_partials, capacity, count_dev,
                                     bin_base, 0, tile_passes, s, false, err_dev);
            }
            StageScope st_(ST_RANGES, s);
            launch_tile_ranges(capacity, count_dev, b.point_keys, keys16, im.ranges, s);
        }
        const bool fwd_depth = in.render_depth && in.camera_type == CAM_PINHOLE;
        const bool fwd_order = render_forward_needs_order(d.T);
        if (fwd_order) { StageScope st_(ST_RANGES, s); launch_tile_order(im.ranges, nullptr, d.T, im.tile_order, s); }
        if (rerun) OMR_HIP(hipMemsetAsync(im.tile_cost, 0, d.T * sizeof(uint32_t), s));
        RenderFwdArgs ra;
        ra.W = in.width; ra.H = in.height; ra.gx = d.gx; ra.gy = d.gy;
        ra.ranges = im.ranges; ra.tile_order = fwd_order ? im.tile_order : nullptr; ra.binning = bin_base; ra.count = count_dev; ra.capacity = capacity;
        ra.splat = g.splat;
        ra.bg = in.background; ra.tile_cost = im.tile_cost; ra.final_T = im.final_T; ra.n_contrib = im.n_contrib;
        ra.max_contrib = im.max_contrib; ra.final_C = im.final_C;
        ra.out_color = in.out_color;
        // lonlat never renders depth (rasterize_points.cu:133-156 passes render_depth to the pinhole path only)
        { StageScope st_(ST_RENDER_FWD, s); launch_render_forward(ra, fwd_depth, s); }
        return OMR_OK;
    };
    if (int e = back_half(cap)) return e;
    if (!known)
        if (int e = wait_count()) return e;
    if (L > cap) {  // the hint was too small: redo the back half at the exact size (outputs are overwritten)
        cap = L;
        rerun = true;
        // the count words were read already: the re-run's emit must not write the pinned slot again (a later
        // forward of this thread on another stream could be reading it by the time this write lands)
        count_words.dst = nullptr;
        rt_add(RS_BACK_HALF_RERUNS, 1);
        if (int e = back_half(cap)) return e;
    }
    hint = L + L / 8 + 4096;
    if (int e = hip_check("emit/sort/render")) return e;
    if (in.num_rendered) *in.num_rendered = (int)L;
    return OMR_OK;
}

struct BackwardIn {
    int camera_type;
    int P, D, M, R;
    const float* background;
    int width, height;
    const float *means3D, *shs, *colors_precomp, *scales;
    float scale_modifier;
    const float *rotations, *cov3D_precomp, *viewmatrix, *projmatrix, *campos;
    float tan_fovx, tan_fovy;
    const int* radii;
    char *geom_buffer, *binning_buffer, *image_buffer;
    const float* dL_dpix;
    float *dL_dmean2D, *dL_dconic, *dL_dopacity, *dL_dcolor, *dL_dmean3D, *dL_dcov3D, *dL_dsh, *dL_dscale, *dL_drot;
    float *dpx_dt, *dpy_dt;
    hipStream_t stream;
};

int backward_impl(const BackwardIn& in)
{
    const hipEvent_t colors_event = t_colors_event;  // omr_backward_colors_event applies to this call only
    t_colors_event = nullptr;
    std::vector<hipEvent_t> chunk_events;  // omr_backward_chunk_events: likewise
    chunk_events.swap(t_chunk_events);
    g_last_error.clear();
    if (in.camera_type != CAM_PINHOLE && in.camera_type != CAM_LONLAT)
        return fail(OMR_ERR_CAMERA_TYPE, "[CudaRasterizer]Invalid camera_type");
    if (in.P < 0 || in.R < 0 || in.width <= 0 || in.height <= 0) return fail(OMR_ERR_INVALID_ARGUMENT, "bad sizes");
    if (in.P == 0) return OMR_OK;
    if (!in.geom_buffer || !in.binning_buffer || !in.image_buffer || !in.dL_dpix)
        return fail(OMR_ERR_INVALID_ARGUMENT, "missing scratch buffer or dL_dpix");
    if (!in.dL_dmean2D || !in.dL_dopacity || !in.dL_dcolor || !in.dL_dmean3D || !in.dL_dcov3D || !in.dL_dscale || !in.dL_drot)
        return fail(OMR_ERR_INVALID_ARGUMENT, "missing gradient output pointer");
    // dL_dsh == NULL with M > 0: not written (omnigs_raster.h; the view-parallel compact exchange rebuilds it)
    if ((in.dpx_dt == nullptr) != (in.dpy_dt == nullptr)) return fail(OMR_ERR_INVALID_ARGUMENT, "dpx_dt / dpy_dt: both or neither");
    const Dims d = dims(in.width, in.height);
    const hipStream_t s = in.stream;
    const size_t P = (size_t)in.P;
    GeomState g;  // as the forward carved it for this view and these inputs (sh_jac is used only if its key matches)
    GeomState::carve(in.geom_buffer, P, &g, row_binning(d.gx, d.gy),
                     sh_jac_stored(in.colors_precomp, in.M, in.shs));
    BinningState b;
    BinningState::carve(in.binning_buffer, (size_t)in.R, d.gx, d.gy, &b);
    ImageState im;
    ImageState::carve(in.image_buffer, d.N, d.T, &im);
    const int* radii = in.radii ? in.radii : geom_internal_radii(in.geom_buffer, P);
    rt_add(RS_BACKWARDS, 1);
    // the forward's back half (emit, tile sort) reports look-back give-ups into counters[3] after the forward
    // returned: read it here, and wait for it only once the whole backward is queued (no GPU bubble)
    HostSlots* hs = host_slots(s);
    if (!hs) return fail(OMR_ERR_HIP, "pinned host memory / event allocation failed");
    hs->words[4] = 0;
    hipError_t rerr;
    HostWords err_words = read_to_host(hs->bwd, g.counters + 3, 1, s, in.R == 0, &rerr);  // carried by backward_schedule
    OMR_HIP(rerr);

    const size_t R = (size_t)in.R;
    char* const lb = in.binning_buffer;  // the L-indexed region (raster_common.h), at offsets of R
    RenderBwdArgs rb;
    rb.W = in.width; rb.H = in.height; rb.gx = d.gx; rb.gy = d.gy;
    rb.ranges = im.ranges; rb.point_list = b.point_list; rb.splat = g.splat; rb.bg = in.background;
    rb.row_first = g.row_first;
    rb.final_T = im.final_T; rb.final_C = im.final_C; rb.n_contrib = im.n_contrib; rb.dL_dpix = in.dL_dpix;
    rb.inst_grad = b.inst_grad;
    rb.row_valid = b.row_valid;
    rb.ckpt = reinterpret_cast<const float4*>(lb + ckpt_offset(R));
    uint2* units = reinterpret_cast<uint2*>(lb + units_offset(R, d.T));
    uint32_t* unit_count = reinterpret_cast<uint32_t*>(lb + unit_words_offset(R, d.T));
    rb.units = units;
    rb.unit_count = unit_count;
    // b.row_valid [R] was zeroed by the forward's render_fwd (row_valid_offset)
    // (tile, depth segment) units, costliest first per XCD share (outside the render_backward stage, so the stage,
    // the bench's roofline duration and the rocprofv3 kernel average all time render_bwd_kernel alone)
    if (R > 0)
        launch_backward_schedule(err_words, im.ranges, im.max_contrib, d.T, reinterpret_cast<uint2*>(lb + units_tmp_offset(R, d.T)),
                                 reinterpret_cast<uint32_t*>(lb + units_tmp_offset(R, d.T) + seg_count(R, d.T) * 8),
                                 units, unit_count, render_backward_needs_order(seg_count(R, d.T)), s);
    {
        StageScope st_(ST_RENDER_BWD, s, true);
        if (R > 0) launch_render_backward(rb, seg_count(R, d.T), s, st_.start(), st_.stop());
    }

    GaussBwdArgs ga;
    ga.P = in.P; ga.D = in.D; ga.M = in.M; ga.W = in.width; ga.H = in.height;
    ga.means3D = in.means3D; ga.radii = radii; ga.shs = in.shs; ga.scales = in.scales; ga.rotations = in.rotations;
    ga.scale_modifier = in.scale_modifier; ga.cov3D_precomp = in.cov3D_precomp; ga.viewmatrix = in.viewmatrix;
    ga.projmatrix = in.projmatrix; ga.campos = in.campos; ga.tan_fovx = in.tan_fovx; ga.tan_fovy = in.tan_fovy;
    ga.focal_y = (float)in.height / (2.0f * in.tan_fovy);
    ga.focal_x = (float)in.width / (2.0f * in.tan_fovx);
    ga.clamped = g.clamped;
    ga.sh_jac = g.sh_jac;
    ga.jac_flag = g.counters + 5;
    ga.row_sums = g.row_sums;
    ga.conic_op = g.conic_op;
    ga.dL_dmean2D = in.dL_dmean2D; ga.dL_dconic = in.dL_dconic; ga.dL_dopacity = in.dL_dopacity; ga.dL_dcolor = in.dL_dcolor;
    ga.dL_dmean3D = in.dL_dmean3D; ga.dL_dcov3D = in.dL_dcov3D; ga.dL_dsh = in.M > 0 ? in.dL_dsh : nullptr;
    ga.dL_dscale = in.dL_dscale; ga.dL_drot = in.dL_drot; ga.dpx_dt = in.dpx_dt; ga.dpy_dt = in.dpy_dt;
    if (!in.shs) ga.shs = nullptr;
    {
        StageScope st_(ST_ROW_SUMS, s);
        launch_row_sums(0, in.P, true, g.row_first, g.tiles_touched, g.huge_list, g.counters + 2, b.inst_grad,
                        b.row_valid, (uint32_t)in.R, g.row_sums, in.dL_dcolor, s);
    }
    if (colors_event) OMR_HIP(hipEventRecord(colors_event, s));  // dL_dcolor is final from here on
    if (chunk_events.empty()) {
        ga.g_begin = 0;
        ga.g_end = in.P;
        StageScope st_(ST_GAUSS_BWD, s, true);
        launch_gaussian_backward(in.camera_type, ga, s, st_.start(), st_.stop());
    } else {  // Gaussian ranges, an event after each: a view-parallel host reduces each range as soon as it is final
        const int nch = (int)chunk_events.size();
        StageScope st_(ST_GAUSS_BWD, s);
        for (int k = 0; k < nch; ++k) {
            ga.g_begin = omr_backward_chunk_begin(in.P, nch, k);
            ga.g_end = omr_backward_chunk_begin(in.P, nch, k + 1);
            launch_gaussian_backward(in.camera_type, ga, s, nullptr, nullptr);
            OMR_HIP(hipEventRecord(chunk_events[k], s));
        }
    }
    if (int e = hip_check("backward")) return e;
    OMR_HIP(timed_wait(hs->bwd, s, RS_BWD_WAIT_NS));
    if (hs->words[4] != 0) {
        rt_add(RS_LOOKBACK_ERRORS, 1);
        return fail(OMR_ERR_HIP, "forward tile sort: a decoupled look-back gave up waiting for a predecessor");
    }
    return OMR_OK;
}

}  // namespace
}  // namespace omr

using namespace omr;

extern "C" {

int omr_abi_version(void) { return OMR_ABI_VERSION; }
void omr_backward_colors_event(void* event) { t_colors_event = static_cast<hipEvent_t>(event); }
void omr_backward_chunk_events(int n, void* const* events)
{
    t_chunk_events.clear();
    for (int k = 0; k < n && events; ++k) t_chunk_events.push_back(static_cast<hipEvent_t>(events[k]));
}
int omr_backward_chunk_begin(int P, int n, int k)
{
    if (n <= 0 || k <= 0) return 0;
    if (k >= n) return std::max(P, 0);
    return (int)((int64_t)std::max(P, 0) * k / n / 256 * 256);  // multiples of 256 (gaussian_bwd's wave layout)
}
const char* omr_last_error(void) { return g_last_error.c_str(); }

int omr_rasterizer_mark_visible(int P, const float* means3D, const float* viewmatrix, const float* projmatrix,
                                bool* present, void* stream)
{
    g_last_error.clear();
    if (P < 0) return fail(OMR_ERR_INVALID_ARGUMENT, "P < 0");
    launch_mark_visible(CAM_PINHOLE, P, means3D, viewmatrix, projmatrix, present, (hipStream_t)stream);
    return hip_check("mark_visible");
}

int omr_lonlat_mark_visible(int P, bool* present, void* stream)
{
    g_last_error.clear();
    if (P < 0) return fail(OMR_ERR_INVALID_ARGUMENT, "P < 0");
    launch_mark_visible(CAM_LONLAT, P, nullptr, nullptr, nullptr, present, (hipStream_t)stream);
    return hip_check("mark_visible");
}

int omr_rasterizer_forward(omr_alloc_fn geometry_alloc, void* geometry_ctx, omr_alloc_fn binning_alloc,
                           void* binning_ctx, omr_alloc_fn image_alloc, void* image_ctx, int P, int D, int M,
                           const float* background, int width, int height, const float* means3D, const float* shs,
                           const float* colors_precomp, const float* opacities, const float* scales,
                           float scale_modifier, const float* rotations, const float* cov3D_precomp,
                           const float* viewmatrix, const float* projmatrix, const float* cam_pos, float tan_fovx,
                           float tan_fovy, bool prefiltered, float* out_color, int* radii, bool render_depth,
                           void* stream, int* num_rendered)
{
    ForwardIn in{CAM_PINHOLE, geometry_alloc, binning_alloc, image_alloc, geometry_ctx, binning_ctx, image_ctx,
                 P, D, M, background, width, height, means3D, shs, colors_precomp, opacities, scales, scale_modifier,
                 rotations, cov3D_precomp, viewmatrix, projmatrix, cam_pos, tan_fovx, tan_fovy, prefiltered,
                 out_color, radii, render_depth, (hipStream_t)stream, num_rendered};
    return forward_impl(in);
}

int omr_lonlat_forward(omr_alloc_fn geometry_alloc, void* geometry_ctx, omr_alloc_fn binning_alloc, void* binning_ctx,
                       omr_alloc_fn image_alloc, void* image_ctx, int P, int D, int M, const float* background,
                       int width, int height, const float* means3D, const float* shs, const float* colors_precomp,
                       const float* opacities, const float* scales, float scale_modifier, const float* rotations,
                       const float* cov3D_precomp, const float* viewmatrix, const float* cam_pos, bool prefiltered,
                       float* out_color, int* radii, void* stream, int* num_rendered)
{
    ForwardIn in{CAM_LONLAT, geometry_alloc, binning_alloc, image_alloc, geometry_ctx, binning_ctx, image_ctx,
                 P, D, M, background, width, height, means3D, shs, colors_precomp, opacities, scales, scale_modifier,
                 rotations, cov3D_precomp, viewmatrix, nullptr, cam_pos, 0.f, 0.f, prefiltered,
                 out_color, radii, false, (hipStream_t)stream, num_rendered};
    return forward_impl(in);
}

int omr_rasterizer_backward(int P, int D, int M, int R, const float* background, int width, int height,
                            const float* means3D, const float* shs, const float* colors_precomp, const float* scales,
                            float scale_modifier, const float* rotations, const float* cov3D_precomp,
                            const float* viewmatrix, const float* projmatrix, const float* campos, float tan_fovx,
                            float tan_fovy, const int* radii, char* geom_buffer, char* binning_buffer,
                            char* image_buffer, const float* dL_dpix, float* dL_dmean2D, float* dL_dconic,
                            float* dL_dopacity, float* dL_dcolor, float* dL_dmean3D, float* dL_dcov3D, float* dL_dsh,
                            float* dL_dscale, float* dL_drot, void* stream)
{
    BackwardIn in{CAM_PINHOLE, P, D, M, R, background, width, height, means3D, shs, colors_precomp, scales,
                  scale_modifier, rotations, cov3D_precomp, viewmatrix, projmatrix, campos, tan_fovx, tan_fovy, radii,
                  geom_buffer, binning_buffer, image_buffer, dL_dpix, dL_dmean2D, dL_dconic, dL_dopacity, dL_dcolor,
                  dL_dmean3D, dL_dcov3D, dL_dsh, dL_dscale, dL_drot, nullptr, nullptr, (hipStream_t)stream};
    return backward_impl(in);
}

int omr_lonlat_backward(int P, int D, int M, int R, const float* background, int width, int height,
                        const float* means3D, const float* shs, const float* colors_precomp, const float* scales,
                        float scale_modifier, const float* rotations, const float* cov3D_precomp,
                        const float* viewmatrix, const float* campos, const int* radii, char* geom_buffer,
                        char* binning_buffer, char* image_buffer, const float* dL_dpix, float* dL_dmean2D,
                        float* dL_dconic, float* dL_dopacity, float* dL_dcolor, float* dL_dmean3D, float* dL_dcov3D,
                        float* dL_dsh, float* dL_dscale, float* dL_drot, float* dpx_dt, float* dpy_dt, void* stream)
{
    BackwardIn in{CAM_LONLAT, P, D, M, R, background, width, height, means3D, shs, colors_precomp, scales,
                  scale_modifier, rotations, cov3D_precomp, viewmatrix, nullptr, campos, 0.f, 0.f, radii,
                  geom_buffer, binning_buffer, image_buffer, dL_dpix, dL_dmean2D, dL_dconic, dL_dopacity, dL_dcolor,
                  dL_dmean3D, dL_dcov3D, dL_dsh, dL_dscale, dL_drot, dpx_dt, dpy_dt, (hipStream_t)stream};
    return backward_impl(in);
}

int omr_sh_grad_from_colors(int P, int D, int M, int nviews, const float* means3D, const float* shs,
                            const float* campos, const float* dL_dcolors, float* dL_dsh, void* stream)
{
    g_last_error.clear();
    if (P < 0 || nviews < 0 || M < 0 || M > 16) return fail(OMR_ERR_INVALID_ARGUMENT, "bad P / M / nviews");
    if (P == 0 || M == 0) return OMR_OK;
    if (!means3D || !shs || !campos || !dL_dcolors || !dL_dsh) return fail(OMR_ERR_INVALID_ARGUMENT, "missing pointer");
    launch_sh_grad_from_colors(P, D, M, nviews, means3D, shs, campos, 3, dL_dcolors, (size_t)P * 3, dL_dsh,
                               (hipStream_t)stream);
    return hip_check("sh_grad_from_colors");
}

int omr_sh_grad_from_colors_packed(int P, int D, int M, int nviews, const float* means3D, const float* shs,
                                   const float* packed, float* dL_dsh, void* stream)
{
    g_last_error.clear();
    if (P < 0 || nviews < 0 || M < 0 || M > 16) return fail(OMR_ERR_INVALID_ARGUMENT, "bad P / M / nviews");
    if (P == 0 || M == 0) return OMR_OK;
    if (!means3D || !shs || !packed || !dL_dsh) return fail(OMR_ERR_INVALID_ARGUMENT, "missing pointer");
    const size_t stride = ((size_t)P + 1) * 3;  // [nviews][P + 1][3]: P colour-gradient rows, then campos
    launch_sh_grad_from_colors(P, D, M, nviews, means3D, shs, packed + (size_t)P * 3, stride, packed, stride, dL_dsh,
                               (hipStream_t)stream);
    return hip_check("sh_grad_from_colors_packed");
}

size_t omr_l1_ssim_scratch_floats(int C, int H, int W)
{
    return (C <= 0 || H <= 0 || W <= 0) ? 0 : l1_ssim_scratch_floats(C, H, W);
}

int omr_l1_ssim_loss(const float* img, const float* gt, int C, int H, int W, float lambda_dssim, float* dL_dimg,
                     float* out3, float* scratch, void* stream)
{
    g_last_error.clear();
    if (C <= 0 || H <= 0 || W <= 0) return fail(OMR_ERR_INVALID_ARGUMENT, "bad C / H / W");
    if (!img || !gt || !dL_dimg || !out3 || !scratch) return fail(OMR_ERR_INVALID_ARGUMENT, "missing pointer");
    launch_l1_ssim(img, gt, C, H, W, lambda_dssim, dL_dimg, out3, scratch, (hipStream_t)stream);
    return hip_check("l1_ssim_loss");
}

static bool aligned16(const void* p) { return ((uintptr_t)p & 15u) == 0; }

// act (4 pointers or NULL): shs, opacity, scales, rotations written from the updated parameters (AdamGroup::act)
static int adam_impl(int P, int Mr, float* const params[6], float* const exp_avg[6], float* const exp_avg_sq[6],
                     const float* const grads[6], int grad_kind, const float lr[6], const int64_t step[6], float beta1,
                     float beta2, float eps, float* const act[4], const DensifyStatsArgs* stats,
                     hipStream_t stream)
{
    g_last_error.clear();
    if (P < 0 || Mr < 0 || Mr > 15) return fail(OMR_ERR_INVALID_ARGUMENT, "bad P / Mr");
    if (grad_kind != OMR_ADAM_RAW_GRADS && grad_kind != OMR_ADAM_RASTER_GRADS)
        return fail(OMR_ERR_INVALID_ARGUMENT, "bad grad_kind");
    if (!params || !exp_avg || !exp_avg_sq || !grads || !lr || !step) return fail(OMR_ERR_INVALID_ARGUMENT, "missing array");
    if ((size_t)P * 3 * (size_t)(Mr + 1) > 0xFFFFFFF0u) return fail(OMR_ERR_INVALID_ARGUMENT, "P too large");
    const uint32_t width[6] = {3u, 3u, 3u * (uint32_t)Mr, 1u, 3u, 4u};
    static const int raster_kind[6] = {ADAM_PLAIN, ADAM_SH_DC, ADAM_SH_REST, ADAM_OPACITY, ADAM_SCALING, ADAM_ROTATION};
    bool active[6];
    for (int k = 0; k < 6; ++k) {
        active[k] = (uint32_t)P * width[k] != 0 && params[k] && grads[k];  // adam.cpp skips parameters without a gradient
        if (!active[k]) continue;
        if (!exp_avg[k] || !exp_avg_sq[k]) return fail(OMR_ERR_INVALID_ARGUMENT, "missing optimizer state");
        const bool gplain = grad_kind == OMR_ADAM_RAW_GRADS || (k != 1 && k != 2);
        if (!aligned16(params[k]) || !aligned16(exp_avg[k]) || !aligned16(exp_avg_sq[k]) || (gplain && !aligned16(grads[k])))
            return fail(OMR_ERR_INVALID_ARGUMENT, "parameter / state / gradient not 16-byte aligned");
        if (step[k] < 1) return fail(OMR_ERR_INVALID_ARGUMENT, "step must be >= 1");
    }
    // the activated outputs: only from the rasterizer's gradients, and only for groups that step (a skipped group's
    // output would be stale); SH needs both f_dc and f_rest (Mr = 0: f_dc alone)
    static const int act_group[4] = {1, 3, 4, 5};
    if (act)
        for (int j = 0; j < 4; ++j) {
            if (!act[j] || P == 0) continue;
            if (grad_kind != OMR_ADAM_RASTER_GRADS)
                return fail(OMR_ERR_INVALID_ARGUMENT, "activated outputs need the rasterizer's gradients (grad_kind 1)");
            if (!active[act_group[j]] || (j == 0 && Mr > 0 && !active[2]))
                return fail(OMR_ERR_INVALID_ARGUMENT, "an activated output of a group that does not step");
            if (!aligned16(act[j])) return fail(OMR_ERR_INVALID_ARGUMENT, "activated output not 16-byte aligned");
        }
    AdamArgs a{};
    a.M = Mr + 1;
    a.beta1 = beta1, a.beta2 = beta2, a.omb1 = (float)(1.0 - (double)beta1), a.omb2 = (float)(1.0 - (double)beta2);
    a.eps = eps;
    // adam.cpp: bias corrections in double, step_size = lr / bias_correction1
    auto consts = [&](int k, float& nss, float& bc2s) {
        const double bc1 = 1.0 - std::pow((double)beta1, (double)step[k]);
        const double bc2 = 1.0 - std::pow((double)beta2, (double)step[k]);
        nss = (float)(-((double)lr[k] / bc1));
        bc2s = (float)std::sqrt(bc2);
    };
    // f_dc + f_rest as one walk over dL_dsh's rows (ADAM_SH_ROWS) whenever both step from the rasterizer's dL_dsh
    // (omr_debug_adam_sh_rows(0) / OMR_ADAM_SH_ROWS=0: the two gathering groups instead, for A/B runs)
    const bool rows = adam_sh_rows_mode().load() != 0 && grad_kind == OMR_ADAM_RASTER_GRADS && Mr > 0 && active[1] &&
                      active[2];
    // without the row walk (A/B switch) the activated SH array is copied from the updated f_dc / f_rest afterwards
    const bool sh_copy_after = act && act[0] && P > 0 && Mr > 0 && !rows;
    for (int k = 0; k < 6; ++k) {
        if (!active[k] || (rows && k == 1)) continue;  // rows: f_dc steps with f_rest's group
        AdamGroup& G = a.group[a.ngroups++];
        G.p = params[k], G.m = exp_avg[k], G.v = exp_avg_sq[k], G.g = grads[k], G.n = (uint32_t)P * width[k];
        G.kind = grad_kind == OMR_ADAM_RAW_GRADS ? ADAM_PLAIN : raster_kind[k];
        consts(k, G.neg_step_size, G.bc2_sqrt);
        for (int j = 0; j < 4; ++j)  // SH (j = 0) on f_dc's group only when Mr = 0: a copy
            if (act && act_group[j] == k && !(j == 0 && sh_copy_after)) G.act = act[j];
        if (rows && k == 2) {
            G.kind = ADAM_SH_ROWS;
            G.act = act ? act[0] : nullptr;
            G.p2 = params[1], G.m2 = exp_avg[1], G.v2 = exp_avg_sq[1];
            consts(1, G.neg_step_size2, G.bc2_sqrt2);
        }
    }
    if (stats && stats->P > 0) {
        if (stats->P != P) return fail(OMR_ERR_INVALID_ARGUMENT, "densification statistics for another P");
        if (!stats->radii || !stats->vgrad || !stats->accum || !stats->denom || !stats->max_radii || stats->vstride < 2)
            return fail(OMR_ERR_INVALID_ARGUMENT, "densification statistics: missing pointer / bad stride");
        a.stats = *stats;
    }
    launch_adam(a, stream);
    if (sh_copy_after) {  // activate_kernel's SH blocks alone (opacity_out NULL), on the parameters Adam just wrote
        ActivateArgs c{};
        c.P = P, c.Mr = Mr, c.f_dc = params[1], c.f_rest = params[2], c.shs = act[0];
        launch_activate(c, stream);
    }
    return hip_check("adam_step");
}

int omr_adam_step(int P, int Mr, float* const params[6], float* const exp_avg[6], float* const exp_avg_sq[6],
                  const float* const grads[6], int grad_kind, const float lr[6], const int64_t step[6], float beta1,
                  float beta2, float eps, void* stream)
{
    return adam_impl(P, Mr, params, exp_avg, exp_avg_sq, grads, grad_kind, lr, step, beta1, beta2, eps, nullptr,
                     nullptr, (hipStream_t)stream);
}

int omr_adam_step_activate(int P, int Mr, float* const params[6], float* const exp_avg[6],
                           float* const exp_avg_sq[6], const float* const grads[6], const float lr[6],
                           const int64_t step[6], float beta1, float beta2, float eps, float* shs, float* opacity,
                           float* scales, float* rotations, const int* radii, const float* viewspace_grad,
                           int viewspace_stride, float* xyz_gradient_accum, float* denom, float* max_radii2D,
                           void* stream)
{
    float* const act[4] = {shs, opacity, scales, rotations};
    DensifyStatsArgs st;
    if (radii) {  // the statistics ride along (omr_densification_stats' arithmetic)
        st.P = P, st.radii = radii, st.vgrad = viewspace_grad, st.vstride = viewspace_stride;
        st.accum = xyz_gradient_accum, st.denom = denom, st.max_radii = max_radii2D;
    }
    return adam_impl(P, Mr, params, exp_avg, exp_avg_sq, grads, OMR_ADAM_RASTER_GRADS, lr, step, beta1, beta2, eps,
                     act, radii ? &st : nullptr, (hipStream_t)stream);
}

int omr_activate(int P, int Mr, const float* const params[6], float* shs, float* opacity, float* scales,
                 float* rotations, void* stream)
{
    g_last_error.clear();
    if (P < 0 || Mr < 0 || Mr > 15) return fail(OMR_ERR_INVALID_ARGUMENT, "bad P / Mr");
    if (P == 0) return OMR_OK;
    if (!params || !params[3] || !params[4] || !params[5] || !opacity || !scales || !rotations ||
        (shs && (!params[1] || (Mr > 0 && !params[2]))))
        return fail(OMR_ERR_INVALID_ARGUMENT, "missing array");
    if (!aligned16(params[5]) || !aligned16(rotations) || (shs && !aligned16(shs)))
        return fail(OMR_ERR_INVALID_ARGUMENT, "rotation / SH arrays not 16-byte aligned");
    if ((size_t)P * 3 * (size_t)(Mr + 1) > 0xFFFFFFF0u) return fail(OMR_ERR_INVALID_ARGUMENT, "P too large");
    ActivateArgs a{};
    a.P = P, a.Mr = Mr;
    a.f_dc = params[1], a.f_rest = params[2], a.opacity = params[3], a.scaling = params[4], a.rotation = params[5];
    a.shs = shs, a.opacity_out = opacity, a.scales_out = scales, a.rotations_out = rotations;
    launch_activate(a, (hipStream_t)stream);
    return hip_check("activate");
}

int omr_densification_stats(int P, const int* radii, const float* viewspace_grad, int viewspace_stride,
                            float* xyz_gradient_accum, float* denom, float* max_radii2D, void* stream)
{
    g_last_error.clear();
    if (P < 0 || viewspace_stride < 2) return fail(OMR_ERR_INVALID_ARGUMENT, "bad P / stride");
    if (P == 0) return OMR_OK;
    if (!radii || !viewspace_grad || !xyz_gradient_accum || !denom || !max_radii2D)
        return fail(OMR_ERR_INVALID_ARGUMENT, "missing pointer");
    launch_densification_stats(P, radii, viewspace_grad, viewspace_stride, xyz_gradient_accum, denom, max_radii2D,
                               (hipStream_t)stream);
    return hip_check("densification_stats");
}

size_t omr_densify_plan_bytes(int P) { return densify_plan_bytes(P); }

int omr_densify_plan(int P, const float* xyz_gradient_accum, const float* denom, const float* scaling,
                     const float* opacity, float max_grad, float min_opacity, float extent, float percent_dense,
                     int max_screen_size, int prune_by_extent, void* plan, int64_t counts[4], void* stream)
{
    g_last_error.clear();
    if (P < 0) return fail(OMR_ERR_INVALID_ARGUMENT, "bad P");
    if (!plan || !counts) return fail(OMR_ERR_INVALID_ARGUMENT, "missing pointer");
    if (P > 0 && (!xyz_gradient_accum || !denom || !scaling || !opacity))
        return fail(OMR_ERR_INVALID_ARGUMENT, "missing pointer");
    hipStream_t s = (hipStream_t)stream;
    launch_densify_plan(P, xyz_gradient_accum, denom, scaling, opacity, max_grad, min_opacity, extent, percent_dense,
                        max_screen_size, prune_by_extent, (char*)plan, s);
    uint4 t;
    OMR_HIP(hipMemcpyAsync(&t, densify_plan_totals(P, (const char*)plan), sizeof(t), hipMemcpyDeviceToHost, s));
    OMR_HIP(hipStreamSynchronize(s));
    counts[0] = (int64_t)t.x + t.y + 2 * (int64_t)t.z;  // P after densify and prune
    counts[1] = t.y;                                     // clones kept
    counts[2] = t.w;                                     // split-selected: rows of normals = 2 * counts[2]
    counts[3] = t.z;                                     // splits kept (each adds two points)
    return hip_check("densify_plan");
}

int omr_densify_apply(int P, int Mr, const void* plan, const float* const params_in[6],
                      const float* const exp_avg_in[6], const float* const exp_avg_sq_in[6], const int32_t* exist_in,
                      const float* normals, float* const params_out[6], float* const exp_avg_out[6],
                      float* const exp_avg_sq_out[6], int32_t* exist_out, void* stream)
{
    g_last_error.clear();
    if (P < 0 || Mr < 0 || Mr > 15) return fail(OMR_ERR_INVALID_ARGUMENT, "bad P / Mr");
    if (P == 0) return OMR_OK;
    if (!plan || !params_in || !params_out) return fail(OMR_ERR_INVALID_ARGUMENT, "missing pointer");
    DensifyIO io{};
    for (int k = 0; k < 6; ++k) {
        if ((!params_in[k] || !params_out[k]) && !(k == 2 && Mr == 0))
            return fail(OMR_ERR_INVALID_ARGUMENT, "missing parameter pointer");
        io.p_in[k] = params_in[k], io.p_out[k] = params_out[k];
        io.m_in[k] = exp_avg_in ? exp_avg_in[k] : nullptr;
        io.v_in[k] = exp_avg_sq_in ? exp_avg_sq_in[k] : nullptr;
        io.m_out[k] = exp_avg_out ? exp_avg_out[k] : nullptr;
        io.v_out[k] = exp_avg_sq_out ? exp_avg_sq_out[k] : nullptr;
    }
    if (exist_out && !exist_in) return fail(OMR_ERR_INVALID_ARGUMENT, "exist_out without exist_in");
    io.exist_in = exist_in, io.exist_out = exist_out;
    io.normals = normals;
    io.Mr = Mr;
    launch_densify_apply(P, (const char*)plan, io, (hipStream_t)stream);
    return hip_check("densify_apply");
}

int omr_reset_opacity(int P, float* opacity, float* exp_avg, float* exp_avg_sq, float ceiling, void* stream)
{
    g_last_error.clear();
    if (P < 0) return fail(OMR_ERR_INVALID_ARGUMENT, "bad P");
    if (P == 0) return OMR_OK;
    if (!opacity) return fail(OMR_ERR_INVALID_ARGUMENT, "missing pointer");
    launch_reset_opacity(P, opacity, exp_avg, exp_avg_sq, ceiling, (hipStream_t)stream);
    return hip_check("reset_opacity");
}

size_t omr_dist2_scratch_bytes(int P) { return P > 0 ? knn_scratch_bytes(P) : 0; }

int omr_dist2(int P, const float* points, float* mean_dists, void* scratch, void* stream)
{
    g_last_error.clear();
    if (P < 0) return fail(OMR_ERR_INVALID_ARGUMENT, "bad P");
    if (P == 0) return OMR_OK;
    if (!points || !mean_dists || !scratch) return fail(OMR_ERR_INVALID_ARGUMENT, "missing pointer");
    launch_knn(P, points, mean_dists, (char*)scratch, (hipStream_t)stream);
    return hip_check("dist2");
}

struct omr_ply {
    PlyFile* f;
};

int omr_ply_open(const char* path, int max_sh_degree, omr_ply** out, int64_t* num_points)
{
    g_last_error.clear();
    if (!path || !out || !num_points) return fail(OMR_ERR_INVALID_ARGUMENT, "missing pointer");
    if (max_sh_degree < 0 || max_sh_degree > 3) return fail(OMR_ERR_INVALID_ARGUMENT, "max_sh_degree must be 0..3");
    std::string err;
    PlyFile* f = ply_open(path, max_sh_degree, err);
    if (!f) return fail(OMR_ERR_INVALID_ARGUMENT, err);
    *out = new omr_ply{f};
    *num_points = ply_num_points(f);
    return OMR_OK;
}

int omr_ply_read(omr_ply* ply, float* const params[6], void* stream)
{
    g_last_error.clear();
    if (!ply || !params) return fail(OMR_ERR_INVALID_ARGUMENT, "missing pointer");
    if (ply_num_points(ply->f) > 0)
        for (int k = 0; k < 6; ++k)
            if (!params[k] && !(k == 2 && ply_rest_coeffs(ply->f) == 0))
                return fail(OMR_ERR_INVALID_ARGUMENT, "missing parameter pointer");
    std::string err;
    if (!ply_read(ply->f, params, (hipStream_t)stream, err)) return fail(OMR_ERR_INVALID_ARGUMENT, err);
    return hip_check("ply_read");
}

void omr_ply_close(omr_ply* ply)
{
    if (!ply) return;
    ply_close(ply->f);
    delete ply;
}

int omr_ply_save(const char* path, int P, int Mr, const float* const params[6], void* stream)
{
    g_last_error.clear();
    if (!path || P < 0 || Mr < 0 || Mr > 15 || !params) return fail(OMR_ERR_INVALID_ARGUMENT, "bad arguments");
    if (P > 0)
        for (int k = 0; k < 6; ++k)
            if (!params[k] && !(k == 2 && Mr == 0)) return fail(OMR_ERR_INVALID_ARGUMENT, "missing parameter pointer");
    std::string err;
    if (!ply_save(path, P, Mr, params, (hipStream_t)stream, err)) return fail(OMR_ERR_INVALID_ARGUMENT, err);
    return hip_check("ply_save");
}

int omr_forward_status(char* geom_buffer, int P, void* stream)
{
    g_last_error.clear();
    if (!geom_buffer || P < 0) return fail(OMR_ERR_INVALID_ARGUMENT, "forward_status: bad geometry buffer");
    GeomState g;
    GeomState::carve(geom_buffer, (size_t)P, &g);
    uint32_t err = 0;
    const hipStream_t s = (hipStream_t)stream;
    OMR_HIP(hipMemcpyAsync(&err, g.counters + 3, sizeof(err), hipMemcpyDeviceToHost, s));
    OMR_HIP(hipStreamSynchronize(s));
    // not counted in RS_LOOKBACK_ERRORS: a backward on the same buffers reports (and counts) the same word
    if (err != 0) return fail(OMR_ERR_HIP, "forward binning: a decoupled look-back gave up waiting for a predecessor");
    return OMR_OK;
}

size_t omr_geometry_bytes(int P)  // the largest geometry buffer a forward of P Gaussians allocates (both optional tails)
{
    return GeomState::carve(nullptr, (size_t)std::max(P, 0), nullptr, true, true);
}

size_t omr_image_bytes(int width, int height)
{
    const Dims d = dims(width, height);
    return ImageState::carve(nullptr, d.N, d.T, nullptr);
}

size_t omr_binning_bytes(int num_rendered, int width, int height)
{
    const Dims d = dims(width, height);
    return BinningState::carve(nullptr, (size_t)std::max(num_rendered, 0), d.gx, d.gy, nullptr);
}

int omr_debug_wave_sum9(const float* in, float* out, void* stream)
{
    g_last_error.clear();
    debug_wave_sum9_kernel<<<1, 64, 0, (hipStream_t)stream>>>(in, out);
    return hip_check("debug_wave_sum9");
}

int omr_debug_wave_sum9_lds(const float* in, float* out, void* stream)
{
    g_last_error.clear();
    debug_wave_sum9_lds_kernel<<<1, 64, 0, (hipStream_t)stream>>>(in, out);
    return hip_check("debug_wave_sum9_lds");
}

int omr_debug_wave_sum9x2(const float* in, float* out, void* stream)
{
    g_last_error.clear();
    debug_wave_sum9x2_kernel<<<1, 64, 0, (hipStream_t)stream>>>(in, out);
    return hip_check("debug_wave_sum9x2");
}

int omr_debug_wave_scans(const uint32_t* in, uint32_t* out, void* stream)
{
    g_last_error.clear();
    debug_wave_scans_kernel<<<1, 64, 0, (hipStream_t)stream>>>(in, out);
    return hip_check("debug_wave_scans");
}


void omr_profile_enable(int on) { g_prof.on = on != 0; }
void omr_profile_set_mask(uint32_t mask) { g_prof.mask = mask; }

void omr_profile_reset(void)
{
    std::lock_guard<std::mutex> lk(g_prof.mu);
    for (auto& r : g_prof.pending) {
        (void)hipEventSynchronize(r.b);
        g_prof.pool.push_back(r.a);
        g_prof.pool.push_back(r.b);
    }
    g_prof.pending.clear();
    for (int i = 0; i < ST_COUNT; ++i) {
        g_prof.total_ms[i] = 0.0;
        g_prof.count[i] = 0;
    }
}

int omr_profile_read(double* total_ms, uint64_t* counts, int n)
{
    std::lock_guard<std::mutex> lk(g_prof.mu);
    for (auto& r : g_prof.pending) {
        (void)hipEventSynchronize(r.b);
        float ms = 0.f;
        if (hipEventElapsedTime(&ms, r.a, r.b) == hipSuccess) {
            g_prof.total_ms[r.stage] += ms;
            g_prof.count[r.stage] += 1;
        }
        g_prof.pool.push_back(r.a);
        g_prof.pool.push_back(r.b);
    }
    g_prof.pending.clear();
    const int m = std::min(n, (int)ST_COUNT);
    for (int i = 0; i < m; ++i) {
        if (total_ms) total_ms[i] = g_prof.total_ms[i];
        if (counts) counts[i] = g_prof.count[i];
    }
    return m;
}

int omr_runtime_stats(uint64_t* out, int n)
{
    const int m = std::min(n, (int)RS_COUNT);
    for (int i = 0; i < m; ++i) out[i] = g_rt[i].load(std::memory_order_relaxed);
    return m;
}

const char* omr_runtime_stat_name(int i) { return (i >= 0 && i < RS_COUNT) ? kRtStatNames[i] : ""; }

void omr_runtime_stats_reset(void)
{
    for (int i = 0; i < RS_COUNT; ++i) g_rt[i].store(0, std::memory_order_relaxed);
}

const char* omr_profile_stage_name(int stage) { return (stage >= 0 && stage < ST_COUNT) ? kStageNames[stage] : ""; }

int omr_debug_point_list(char* binning_buffer, int R, int width, int height, uint32_t* dst, void* stream)
{
    g_last_error.clear();
    if (R <= 0) return OMR_OK;
    const Dims d = dims(width, height);
    BinningState b;
    BinningState::carve(binning_buffer, (size_t)R, d.gx, d.gy, &b);
    // the Gaussian indices alone (entries carry the instance's band mask in their top bits, raster_common.h)
    debug_point_ids_kernel<<<div_up((size_t)R, 256), 256, 0, (hipStream_t)stream>>>(b.point_list, (size_t)R, dst);
    return hip_check("debug_point_list");
}

int omr_debug_point_list_raw(char* binning_buffer, int R, int width, int height, uint32_t* dst, void* stream)
{
    g_last_error.clear();
    if (R <= 0) return OMR_OK;
    const Dims d = dims(width, height);
    BinningState b;
    BinningState::carve(binning_buffer, (size_t)R, d.gx, d.gy, &b);
    OMR_HIP(hipMemcpyAsync(dst, b.point_list, (size_t)R * sizeof(uint32_t), hipMemcpyDeviceToDevice,
                           (hipStream_t)stream));
    return hip_check("debug_point_list_raw");
}

int omr_debug_ranges(char* image_buffer, int width, int height, uint32_t* dst, void* stream)
{
    g_last_error.clear();
    const Dims d = dims(width, height);
    ImageState im;
    ImageState::carve(image_buffer, d.N, d.T, &im);
    OMR_HIP(hipMemcpyAsync(dst, im.ranges, d.T * sizeof(uint2), hipMemcpyDeviceToDevice, (hipStream_t)stream));
    return OMR_OK;
}

int omr_debug_image_state(char* image_buffer, int width, int height, float* final_T, uint32_t* n_contrib, void* stream)
{
    g_last_error.clear();
    const Dims d = dims(width, height);
    ImageState im;
    ImageState::carve(image_buffer, d.N, d.T, &im);
    OMR_HIP(hipMemcpyAsync(final_T, im.final_T, d.N * sizeof(float), hipMemcpyDeviceToDevice, (hipStream_t)stream));
    OMR_HIP(hipMemcpyAsync(n_contrib, im.n_contrib, d.N * sizeof(uint32_t), hipMemcpyDeviceToDevice, (hipStream_t)stream));
    return OMR_OK;
}

int omr_debug_tile_cost(char* image_buffer, int width, int height, uint32_t* dst, void* stream)
{
    g_last_error.clear();
    const Dims d = dims(width, height);
    ImageState im;
    ImageState::carve(image_buffer, d.N, d.T, &im);
    OMR_HIP(hipMemcpyAsync(dst, im.tile_cost, d.T * sizeof(uint32_t), hipMemcpyDeviceToDevice, (hipStream_t)stream));
    return OMR_OK;
}

int omr_debug_counters(char* geom_buffer, int P, uint32_t* dst, void* stream)
{
    g_last_error.clear();
    GeomState g;
    GeomState::carve(geom_buffer, (size_t)std::max(P, 0), &g);
    OMR_HIP(hipMemcpyAsync(dst, g.counters, 8 * sizeof(uint32_t), hipMemcpyDeviceToDevice, (hipStream_t)stream));
    return OMR_OK;
}

int omr_debug_depth_sort_mode(int mode)
{
    if (mode < 0 || mode > 3) {
        fail(OMR_ERR_INVALID_ARGUMENT, "depth sort mode: 0 (by size and camera type), 1, 2, 3");
        return -1;
    }
    const int old = depth_sort_mode().exchange(mode);
    return old;
}

int omr_debug_binning_mode(int mode)
{
    if (mode < 0 || mode > 2) {
        fail(OMR_ERR_INVALID_ARGUMENT, "binning mode: 0 (by view), 1 (rows), 2 (sort)");
        return -1;
    }
    return binning_mode().exchange(mode);
}

int omr_debug_ssim_mode(int mode)
{
    if (mode < 0 || mode > 2) {
        fail(OMR_ERR_INVALID_ARGUMENT, "ssim mode: 0 (by image size), 1 (tiled), 2 (streaming)");
        return -1;
    }
    return ssim_debug_mode(mode);
}

int omr_debug_bwd_bands(int mode)
{
    if (mode != 0 && mode != 2 && mode != 4) {
        fail(OMR_ERR_INVALID_ARGUMENT, "render backward bands per wave: 0 (by view), 2 or 4");
        return -1;
    }
    return bwd_bands_mode(mode);
}

int omr_debug_adam_sh_rows(int enabled)
{
    if (enabled < 0 || enabled > 1) {
        fail(OMR_ERR_INVALID_ARGUMENT, "adam SH rows: 0 (gathering groups) or 1 (row walk)");
        return -1;
    }
    return adam_sh_rows_mode().exchange(enabled);
}

int omr_debug_set_sh_jac(char* geom_buffer, int P, int enabled, void* stream)
{
    g_last_error.clear();
    GeomState g;
    GeomState::carve(geom_buffer, (size_t)std::max(P, 0), &g);
    // preprocess writes the forward's key to counters[5] and [6]; clearing zeroes [5] only, setting copies [6] back,
    // so any sequence of clears and sets restores the forward's own key
    if (enabled) {
        OMR_HIP(hipMemcpyAsync(g.counters + 5, g.counters + 6, sizeof(uint32_t), hipMemcpyDeviceToDevice,
                               (hipStream_t)stream));
    } else {
        OMR_HIP(hipMemsetAsync(g.counters + 5, 0, sizeof(uint32_t), (hipStream_t)stream));
    }
    OMR_HIP(hipStreamSynchronize((hipStream_t)stream));
    return OMR_OK;
}

int omr_debug_geometry(char* geom_buffer, int P, float* means2D, float* conic_opacity, float* rgb, float* depths,
                       uint32_t* tiles_touched, void* stream)
{
    g_last_error.clear();
    if (P <= 0) return OMR_OK;
    GeomState g;
    GeomState::carve(geom_buffer, (size_t)P, &g);
    const hipStream_t s = (hipStream_t)stream;
    // strided copies out of the 64-B render records (raster_common.h)
    const size_t pitch = SPLAT_F4 * sizeof(float4);
    const char* rec = reinterpret_cast<const char*>(g.splat);
    auto col = [&](void* dst, size_t off, size_t bytes) {
        return hipMemcpy2DAsync(dst, bytes, rec + off, pitch, bytes, P, hipMemcpyDeviceToDevice, s);
    };
    if (means2D) OMR_HIP(col(means2D, 0, 2 * sizeof(float)));
    if (conic_opacity) OMR_HIP(col(conic_opacity, sizeof(float4), sizeof(float4)));
    if (rgb) OMR_HIP(col(rgb, 2 * sizeof(float4), 3 * sizeof(float)));
    if (depths) OMR_HIP(col(depths, 2 * sizeof(float), sizeof(float)));
    if (tiles_touched) OMR_HIP(hipMemcpyAsync(tiles_touched, g.tiles_touched, P * sizeof(uint32_t), hipMemcpyDeviceToDevice, s));
    return OMR_OK;
}

}  // extern "C"
