// sort.hip — binning for the gfx950 rasterizer: u32 scan, stable LSD radix sort, instance emission, tile ranges.
//
// What it replaces: cub::DeviceScan::InclusiveSum + duplicateWithKeys + cub::DeviceRadixSort::SortPairs on
// 64-bit (tile << 32 | depth_bits) keys over [0, 32 + getHigherMsb(T)) + identifyTileRanges
// (cuda_rasterizer/rasterizer_impl.cu:94-167, :622-679).
//
// The reference's result is the stable order (tile, depth_bits, Gaussian index) of all Gaussian x tile
// instances. We produce the same permutation with far fewer key bytes moved:
//   1. stable radix sort of the P Gaussians by depth bits (4 x 8-bit passes over P, not over L instances);
//   2. inclusive scan of tiles_touched in that depth order -> emission slots, num_rendered;
//   3. emit instances in depth order (tile id + Gaussian index, 8 B per instance);
//   4. stable radix sort of the instances by tile id only: ceil(getHigherMsb(T) / 8) passes (2 at <= 64k tiles)
//      instead of ceil((32 + getHigherMsb(T)) / 8) = 6 passes over 12-B pairs.
// Stability of both sorts makes the result bit-identical to the reference permutation.
//
// MI355X notes: 256-thread blocks own 4096-key tiles; digits are ranked inside a wave by 8 ballots
// (wave64 match-any), across the 4 waves of a block through LDS, and across blocks either through a scanned
// [digit][block] histogram (upsweep / scan / downsweep launches per pass) or, for sorts of at most OS_MAX_BLOCKS
// tiles, through a decoupled look-back inside one launch per pass (onesweep_kernel). Either way every key's
// destination follows from counts alone, so the permutation is deterministic.
#include <algorithm>
#include <utility>

#include "kernels.h"

namespace omr {

namespace {

__device__ __forceinline__ uint32_t wave_inclusive_scan(uint32_t x) { return wave_incl_sum_u32(x); }

// block-wide exclusive scan of one value per thread (THREADS threads); returns the block total via *total
template <int THREADS = SCAN_THREADS>
__device__ __forceinline__ uint32_t block_exclusive_scan(uint32_t x, uint32_t* s_wave, uint32_t* total)
{
    const uint32_t lane = lane_id();
    const uint32_t w = threadIdx.x >> 6;
    const uint32_t inc = wave_inclusive_scan(x);
    if (lane == 63) s_wave[w] = inc;
    __syncthreads();
    uint32_t wave_off = 0, tot = 0;
#pragma unroll
    for (int k = 0; k < THREADS / 64; ++k) {
        const uint32_t v = s_wave[k];
        if ((uint32_t)k < w) wave_off += v;
        tot += v;
    }
    __syncthreads();
    *total = tot;
    return wave_off + inc - x;
}

// ---- decoupled look-back (single-launch scans) -------------------------------------------------------------
// Tiles are handed out by a ticket; a tile publishes its total (AGG), looks back over its predecessors with one
// wave, 64 tiles per round trip, until it meets an inclusive prefix (PRE), then publishes its own. 64-bit status
// words, flag in bits 62-63, zeroed before the launch.
// The radix ranks take each round's digit peers from ballot matches (wave_match_digit). The binning scatters'
// LDS OR peer tables (raster_common.h: wave_peer_masks) measured slower here (interleaved A/B,
// profiles/r04i_ab_{A,C,E}.txt: C 0.0801 vs 0.0793 ms, E 0.189 vs 0.180 ms, A equal; the code is in
// profiles/r04_pruned_experiments.patch).
#ifndef OMR_LB_SPIN_MAX
#define OMR_LB_SPIN_MAX (1u << 20)
#endif
constexpr uint32_t LB_SPIN_MAX = OMR_LB_SPIN_MAX;  // polls of one status word before a look-back gives up and sets the
                                                   // error word (capi.hip reports it as OMR_ERR_HIP; a test build shrinks it)
constexpr uint64_t SLB_AGG = 1ull << 62, SLB_PRE = 2ull << 62, SLB_VAL = SLB_AGG - 1;

// lane `src` (wave-uniform) of a 64-bit value: two v_readlane, no LDS crossbar
__device__ __forceinline__ uint64_t readlane_u64(uint64_t v, uint32_t src)
{
    const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)v, (int)src);
    const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(v >> 32), (int)src);
    return ((uint64_t)hi << 32) | lo;
}
// Sum over the wave on every lane, by DPP inside each 16-lane row (quad_perm xor1 / xor2, row_ror 4 / 8) and
// v_permlane16/32_swap across rows (as tile_wave.h: wave_max_u32): no ds_bpermute round trips on the look-back's path
template <int CTRL>
__device__ __forceinline__ uint64_t add_dpp_u64(uint64_t v)
{
    const uint32_t lo = (uint32_t)__builtin_amdgcn_mov_dpp((int)(uint32_t)v, CTRL, 0xf, 0xf, true);
    const uint32_t hi = (uint32_t)__builtin_amdgcn_mov_dpp((int)(uint32_t)(v >> 32), CTRL, 0xf, 0xf, true);
    return v + (((uint64_t)hi << 32) | lo);
}
__device__ __forceinline__ uint64_t wave_sum_u64(uint64_t v)
{
    v = add_dpp_u64<0xb1>(v);   // quad_perm [1,0,3,2]
    v = add_dpp_u64<0x4e>(v);   // quad_perm [2,3,0,1]
    v = add_dpp_u64<0x124>(v);  // row_ror:4
    v = add_dpp_u64<0x128>(v);  // row_ror:8
    uint32_t alo = (uint32_t)v, blo = alo, ahi = (uint32_t)(v >> 32), bhi = ahi;
    asm volatile("s_nop 1\n\tv_permlane16_swap_b32 %0, %1" : "+v"(alo), "+v"(blo));
    asm volatile("s_nop 1\n\tv_permlane16_swap_b32 %0, %1" : "+v"(ahi), "+v"(bhi));
    v = (((uint64_t)ahi << 32) | alo) + (((uint64_t)bhi << 32) | blo);
    alo = (uint32_t)v, blo = alo, ahi = (uint32_t)(v >> 32), bhi = ahi;
    asm volatile("s_nop 1\n\tv_permlane32_swap_b32 %0, %1" : "+v"(alo), "+v"(blo));
    asm volatile("s_nop 1\n\tv_permlane32_swap_b32 %0, %1" : "+v"(ahi), "+v"(bhi));
    return (((uint64_t)ahi << 32) | alo) + (((uint64_t)bhi << 32) | blo);
}

// Called by all 64 lanes of one wave of tile vb: publishes `total`, returns the exclusive prefix of the tile (on every
// lane) and publishes the inclusive one. A predecessor that never publishes ends the wait after LB_SPIN_MAX polls with the
// error word set (no hang).
__device__ uint64_t wave_lookback(uint64_t* status, uint32_t vb, uint32_t total, uint32_t lane, uint32_t* err)
{
    if (vb == 0) {
        if (lane == 0) __hip_atomic_store(&status[0], SLB_PRE | total, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        return 0;
    }
    if (lane == 0) __hip_atomic_store(&status[vb], SLB_AGG | total, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    uint64_t excl = 0;
    uint32_t j = vb, spins = 0;  // next predecessor to read is j - 1 - lane
    while (true) {
        const uint64_t st = j > lane ? __hip_atomic_load(&status[j - 1 - lane], __ATOMIC_RELAXED,
                                                         __HIP_MEMORY_SCOPE_AGENT)
                                     : SLB_PRE;  // never reached: tile 0 publishes PRE
        const uint64_t stop = __ballot((st & ~SLB_VAL) != SLB_AGG);  // PRE or not yet published
        const uint32_t k = stop ? (uint32_t)__builtin_ctzll(stop) : 64u;
        excl += wave_sum_u64(lane < k || (lane == k && (st & SLB_PRE)) ? (st & SLB_VAL) : 0ull);
        if (k < 64u && (readlane_u64(st, k) & SLB_PRE)) break;
        if (k == 0 && ++spins > LB_SPIN_MAX) {
            if (lane == 0) atomicOr(err, 1u);
            break;
        }
        if (k == 0) __builtin_amdgcn_s_sleep(1);
        j -= k;
    }
    if (lane == 0) __hip_atomic_store(&status[vb], SLB_PRE | (excl + total), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    return excl;
}

// ---- the forward's scans of tiles_touched (and the rect rows), in one launch -------------------------------------
// row_first = exclusive scan in Gaussian INDEX order: the first gradient row of each Gaussian. The backward numbers
//             its per-instance gradient rows this way (render_bwd.hip), so the 64 Gaussians of a wave own one
//             contiguous span of rows when their sums are taken (gaussian_bwd.hip: row_sum_kernel); its total is
//             num_rendered;
// sort path (rects == NULL): offsets = inclusive scan of tiles_touched in depth order (gather by `order`): the
//             emission slots (emit_kernel);
// row path (rects != NULL; bin.hip): drect = the rect words in depth order, row_offsets = inclusive scan of their row
//             counts in depth order: the row binning's slots, their total M in count_out[4]; and desc_r, the owners of
//             every BIN_CHUNK-slot chunk: the rank holding the chunk's first slot (x) and its last (y) — each rank
//             covers at most one chunk start (rows <= BIN_MAX_GRID < BIN_CHUNK) and writes the words it decides.
// The sequences have the same tile structure: each 4096-item tile scans them in LDS, and its waves 0 / 1 find the
// exclusive prefixes by decoupled look-back at the same time (status_a: depth order, status_i: index order; ticket,
// error word: scan2_status_words(n), zeroed by preprocess). The kernel also lists the Gaussians with more than
// ROW_SUM_HUGE tiles (huge_list, in no particular order), whose row sums take a whole workgroup.
__global__ __launch_bounds__(SCAN_THREADS) void scan2_lookback_kernel(const uint32_t* in, const uint2* rects,
                                                                      const uint32_t* order, size_t n,
                                                                      uint64_t* status_a, uint64_t* status_i,
                                                                      uint32_t* ticket, uint32_t* err,
                                                                      uint32_t* offsets, uint32_t* row_first,
                                                                      uint32_t* row_offsets, uint2* drect,
                                                                      uint32_t* desc_r, uint32_t* huge_list,
                                                                      uint32_t* huge_count, uint32_t* count_out,
                                                                      const uint32_t* nvis)
{
    __shared__ uint32_t s_a[SCAN_TILE + SCAN_TILE / 32];  // depth order: tiles (sort path) or rows (row path)
    __shared__ uint32_t s_i[SCAN_TILE + SCAN_TILE / 32];  // +1 pad per 32 to break the 16-stride conflicts
    __shared__ uint32_t s_wave[SCAN_THREADS / 64];
    __shared__ uint32_t s_vb, s_huge, s_huge_base;
    __shared__ uint32_t s_excl[2];
    const uint32_t tid = threadIdx.x, lane = tid & 63u;
    const bool rows = rects != nullptr;  // launch-uniform
    if (tid == 0) {
        s_vb = atomicAdd(ticket, 1u);
        s_huge = 0;
    }
    __syncthreads();
    const uint32_t vb = s_vb;
    const size_t base = (size_t)vb * SCAN_TILE;
    auto pad = [](uint32_t i) { return i + (i >> 5); };
    constexpr uint32_t ROWS_MASK = (1u << RECT_ROWS_BITS) - 1u;
    // a depth sort whose look-back gave up may leave `order` partly unwritten: never gather through it then
    const bool order_ok = __hip_atomic_load(err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == 0u;
    // depth ranks past n_a hold culled Gaussians (nvis: the culled-aside depth sort's visible count), which own no
    // tiles and no rows: no order load or gather for them, and on the row path no drect / row_offsets word either (the
    // row binning reads those only at owners of row slots, all visible)
    const size_t n_a = nvis ? min((size_t)*nvis, n) : n;
#pragma unroll
    for (int k = 0; k < SCAN_ITEMS; ++k) {
        const uint32_t li = k * SCAN_THREADS + tid;
        const size_t i = base + li;
        const uint32_t o = i < n_a && order_ok ? order[i] : 0u;
        if (rows) {
            // the one random gather of the forward scans: a second one measured +79 us at config E (139 -> 218 us)
            const uint2 rw = i < n_a && order_ok ? rects[o] : make_uint2(0u, 0u);
            if (i < n_a) drect[i] = rw;
            s_a[pad(li)] = rw.x & ROWS_MASK;
        } else {
            s_a[pad(li)] = i < n_a && order_ok ? in[o] : 0u;
        }
        s_i[pad(li)] = i < n ? in[i] : 0u;
    }
    // the rows of the next tile's first rank, which the tile's last rank needs for its chunk owner word: gathered now,
    // behind the loads above, instead of as two dependent round trips at the end of the kernel's chain
    uint32_t next_tile_rows = 0;
    if (rows && tid == SCAN_THREADS - 1 && base + SCAN_TILE < n_a && order_ok)
        next_tile_rows = rects[order[base + SCAN_TILE]].x & ROWS_MASK;
    __syncthreads();
    uint32_t va[SCAN_ITEMS], vi[SCAN_ITEMS];
    uint32_t sum_a = 0, sum_i = 0;
#pragma unroll
    for (int k = 0; k < SCAN_ITEMS; ++k) {
        va[k] = s_a[pad(tid * SCAN_ITEMS + k)];
        vi[k] = s_i[pad(tid * SCAN_ITEMS + k)];
        sum_a += va[k];
        sum_i += vi[k];
    }
    uint32_t total_a, total_i;
    uint32_t run_a = block_exclusive_scan(sum_a, s_wave, &total_a);
    uint32_t run_i = block_exclusive_scan(sum_i, s_wave, &total_i);
    if (tid < 128u) {  // wave 0: depth order, wave 1: index order
        const uint32_t wv = tid >> 6;
        const uint64_t excl = wave_lookback(wv == 0 ? status_a : status_i, vb, wv == 0 ? total_a : total_i, lane, err);
        if (lane == 0) s_excl[wv] = (uint32_t)excl;
    }
    // the tile's huge Gaussians get consecutive list slots: LDS ranks, one global reservation per tile
    uint32_t hrank[SCAN_ITEMS];
#pragma unroll
    for (int k = 0; k < SCAN_ITEMS; ++k) {
        const uint32_t li = k * SCAN_THREADS + tid;
        hrank[k] = base + li < n && s_i[pad(li)] > ROW_SUM_HUGE ? atomicAdd(&s_huge, 1u) : 0xFFFFFFFFu;
    }
    __syncthreads();
    if (tid == 0) s_huge_base = s_huge ? atomicAdd(huge_count, s_huge) : 0u;
    run_a += s_excl[0];
    run_i += s_excl[1];
#pragma unroll
    for (int k = 0; k < SCAN_ITEMS; ++k) {
        run_a += va[k];  // inclusive
        s_a[pad(tid * SCAN_ITEMS + k)] = run_a;
        s_i[pad(tid * SCAN_ITEMS + k)] = run_i;  // exclusive
        run_i += vi[k];
    }
    __syncthreads();
#pragma unroll
    for (int k = 0; k < SCAN_ITEMS; ++k) {
        const uint32_t li = k * SCAN_THREADS + tid;
        const size_t i = base + li;
        if (i >= n) continue;
        const uint32_t ex_i = s_i[pad(li)];
        row_first[i] = ex_i;
        if (i == n - 1) count_out[0] = s_excl[1] + total_i;  // num_rendered next to the flag words the host reads
        if (hrank[k] != 0xFFFFFFFFu) huge_list[s_huge_base + hrank[k]] = (uint32_t)i;
        const uint32_t incl = s_a[pad(li)];
        if (!rows) {
            offsets[i] = incl;
            if (i == n - 1) count_out[4] = 0u;  // no row slots on this path
            continue;
        }
        if (i == n - 1) count_out[4] = incl;  // M, the row binning's slot count
        if (i >= n_a) continue;  // culled: no rows
        row_offsets[i] = incl;
        // li == 0 is thread 0's first item in both layouts: its own rows are va[0]
        const uint32_t start = li == 0 ? incl - va[0] : s_a[pad(li - 1)];
        if (incl == start) continue;  // no rows (culled: ranked last)
        const uint32_t r = (uint32_t)i;
        const uint32_t kk = (start + BIN_CHUNK - 1) / BIN_CHUNK;  // the first chunk start at or after `start`
        if (kk * BIN_CHUNK < incl) {
            desc_r[2 * kk] = r;  // first owner of chunk kk
            if (kk > 0) desc_r[2 * (kk - 1) + 1] = start < kk * BIN_CHUNK ? r : r - 1;  // last owner of chunk kk - 1
        }
        // the last rank with rows owns the last slot (culled ranks, all rowless, come after every visible one)
        uint32_t next_rows;
        if (i + 1 >= n) next_rows = 0;
        else if (li + 1 < SCAN_TILE) next_rows = s_a[pad(li + 1)] - incl;
        else next_rows = next_tile_rows;  // tid == SCAN_THREADS - 1, k == SCAN_ITEMS - 1
        if (next_rows == 0) desc_r[2 * ((incl - 1) / BIN_CHUNK) + 1] = r;
    }
}

// Exclusive scan of a u32 array in ONE launch, for the [digit][block] histograms of the large sorts (the 3-launch
// reduce / partials / downsweep scan before) and the row binning (bin.hip); status / ticket zeroed by the kernel
// before. Persistent: each block takes tickets (tile numbers, in dispatch order) until they run past the live tiles, so
// a grid capped at SCAN_GRID_MAX blocks serves any length and a capacity-sized scan costs no dispatch of dead blocks
// (a tile looks back only at lower tickets, held by blocks already running: no block waits on one not yet resident).
// n_dev (may be NULL): a device word with the live length (<= n). mask: applied to every input word.
__global__ __launch_bounds__(SCAN_THREADS) void scan_lookback_kernel(const uint32_t* in, uint32_t* out, size_t n,
                                                                     const uint32_t* n_dev, uint64_t* status,
                                                                     uint32_t* ticket, uint32_t* err,
                                                                     uint32_t mask = 0xFFFFFFFFu)
{
    __shared__ uint32_t s_data[SCAN_TILE + SCAN_TILE / 32];
    __shared__ uint32_t s_wave[SCAN_THREADS / 64];
    __shared__ uint32_t s_vb;
    __shared__ uint64_t s_excl;
    const uint32_t tid = threadIdx.x, lane = tid & 63u;
    if (n_dev) n = min(n, (size_t)*n_dev);
    const uint32_t ntiles = max(1u, (uint32_t)((n + SCAN_TILE - 1) / SCAN_TILE));  // tile 0 runs for n = 0 (publishes 0)
    if (blockIdx.x >= ntiles) return;
    auto pad = [](uint32_t i) { return i + (i >> 5); };
    while (true) {
        if (tid == 0) s_vb = atomicAdd(ticket, 1u);
        __syncthreads();
        const uint32_t vb = s_vb;
        if (vb >= ntiles) return;  // block-uniform
        const size_t base = (size_t)vb * SCAN_TILE;
#pragma unroll
        for (int k = 0; k < SCAN_ITEMS; ++k) {
            const uint32_t li = k * SCAN_THREADS + tid;
            const size_t i = base + li;
            s_data[pad(li)] = i < n ? in[i] & mask : 0u;
        }
        __syncthreads();
        uint32_t v[SCAN_ITEMS];
        uint32_t sum = 0;
#pragma unroll
        for (int k = 0; k < SCAN_ITEMS; ++k) {
            v[k] = s_data[pad(tid * SCAN_ITEMS + k)];
            sum += v[k];
        }
        uint32_t total;
        const uint32_t run0 = block_exclusive_scan(sum, s_wave, &total);
        if (tid < 64) {  // wave 0: publish, look back, publish the inclusive prefix
            const uint64_t excl = wave_lookback(status, vb, total, lane, err);
            if (tid == 0) s_excl = excl;
        }
        __syncthreads();
        uint32_t run = (uint32_t)s_excl + run0;
#pragma unroll
        for (int k = 0; k < SCAN_ITEMS; ++k) {
            s_data[pad(tid * SCAN_ITEMS + k)] = run;
            run += v[k];
        }
        __syncthreads();
#pragma unroll
        for (int k = 0; k < SCAN_ITEMS; ++k) {
            const uint32_t li = k * SCAN_THREADS + tid;
            const size_t i = base + li;
            if (i < n) out[i] = s_data[pad(li)];
        }
        __syncthreads();  // s_data and s_vb are rewritten by the next tile
    }
}

// sorts of at most this many 4096-item blocks (the depth sort up to 2M Gaussians) let each downsweep block derive
// its digit offsets from the raw histogram: <= 512 KiB of L2 reads per block instead of three scan launches
constexpr uint32_t SELF_SCAN_MAX_BLOCKS = 512;
#ifndef OMR_SORT_THREADS_LARGE
#define OMR_SORT_THREADS_LARGE 512
#endif
#ifndef OMR_SORT_ITEMS_LARGE
#define OMR_SORT_ITEMS_LARGE (8192 / OMR_SORT_THREADS_LARGE)
#endif
#ifndef OMR_SORT_LARGE_MIN
#define OMR_SORT_LARGE_MIN (1u << 25)
#endif
constexpr int SORT_THREADS_LARGE = OMR_SORT_THREADS_LARGE;  // block size of the multi-launch passes of large sorts
constexpr int SORT_ITEMS_LARGE = OMR_SORT_ITEMS_LARGE;      // items per thread there (8192-key tiles)
constexpr size_t SORT_LARGE_MIN = OMR_SORT_LARGE_MIN;
// block shape of the multi-launch passes below the large-sort threshold: SORT_TILE (4096) keys either way
#ifndef OMR_SORT_THREADS_S
#define OMR_SORT_THREADS_S 512
#endif
constexpr int SORT_THREADS_S = OMR_SORT_THREADS_S;
constexpr int SORT_ITEMS_S = SORT_TILE / SORT_THREADS_S;
// 16-bit keys take the large tiles from 4 M keys on (config C's 7.9 M-key tile sort: 0.1315 -> 0.1217 ms; with
// 32-bit keys 8192-key tiles are slower there, 0.152 vs 0.137 ms)
#ifndef OMR_SORT_LARGE_MIN16
#define OMR_SORT_LARGE_MIN16 (1u << 22)
#endif
constexpr size_t SORT_LARGE_MIN16 = OMR_SORT_LARGE_MIN16;

// ---- radix sort ------------------------------------------------------------------------------------------
// element count: the host's n, or the device count word (binning, capi.hip; raster_common.h: binning_count), which
// reads as 0 when the count is past the capacity (the host re-runs the back half at the exact size) or when a
// look-back has given up (the call fails; nothing downstream touches possibly corrupt offsets or permutations)
__device__ __forceinline__ size_t live_count(size_t n, const uint32_t* count)
{
    return count ? binning_count(count, n) : n;
}

// ---- the depth sort's digits (depth_sort below) -----------------------------------------------------------------
// The culled Gaussians' keys (0xFFFFFFFF) only need to end up behind the visible ones: they own no tiles, so nothing
// downstream depends on their order. The depth keys are float bits of positive depths (bit 31 clear), so 31 bits
// order the visible ones:
//   pass 0: all P keys; digit = bits 0..6 of a visible key, bucket 128 for a culled one: the pass moves the culled
//           Gaussians straight into their final places [nvis, P) of the result (index order) and the visible ones
//           into [0, nvis); passes 1..3 take nvis from their digit totals (onesweep) or from DepthPass::words[0],
//           which block 0 of pass 0's downsweep sets to the start of bucket 128 (upsweep / scan / downsweep);
//   passes 1..3: the nvis visible keys alone, bits [8p - 1, 8p + 7): 8-bit digits as the plain sort's.
// At a frustum that culls most of a scene (config E pinhole: 88 %) passes 1..3 move an eighth of the keys.
// Stable passes order the visible keys exactly as the 32-bit key sort does, ties in index order.
// words[3] stays 0 (zeroed before the sort), so binning_count (live_count) reads nvis from the words.
constexpr uint32_t DEPTH_CULLED_BUCKET = 128;
constexpr int DEPTH_PASSES = 4;
__device__ __forceinline__ uint32_t depth_digit(uint32_t k, int pass)
{
    if (pass == 0) return k == 0xFFFFFFFFu ? DEPTH_CULLED_BUCKET : (k & 127u);
    return (k >> (8 * pass - 1)) & (RADIX - 1u);
}
// one launch of a depth-sort pass: the pass index, the words, and where the permutation goes (the last pass writes
// only it, no keys; pass 0 the culled Gaussians' entries)
struct DepthPass {
    int pass = -1;  // < 0: a plain LSD pass (digit = bits [shift, shift + 8) of the key)
    uint32_t* words = nullptr;
    uint32_t* vals_final = nullptr;
};

// BLOCK_MAJOR: hist[block][digit] (read back by the self-scanning downsweep of small sorts); else hist[digit][block].
// Key arrays are 16-B aligned (Carver) for the 16-B loads.
// DEPTH: a depth-sort pass (dp: DepthPass); its digits
template <typename K, bool BLOCK_MAJOR, int ITEMS, int THREADS, bool DEPTH = false>
__global__ __launch_bounds__(THREADS) void radix_upsweep_kernel(const K* keys, size_t n_cap,
                                                                     const uint32_t* count, int shift, uint32_t* hist,
                                                                     uint32_t nblocks, uint32_t* zero, uint32_t nzero,
                                                                     DepthPass dp = {})
{
    constexpr int TILE_N = THREADS * ITEMS;
    constexpr uint32_t NR = RADIX;
    {   // the look-back words of the histogram scan that follows (scan_lookback_kernel)
        const uint32_t z = blockIdx.x * THREADS + threadIdx.x;
        if (z < nzero) zero[z] = 0u;
    }
    constexpr bool depth = DEPTH;
    const size_t n = live_count(n_cap, count);
    static_assert(THREADS % NR == 0, "thread = digit phases");
    __shared__ uint32_t s_hist[NR];
    if (threadIdx.x < NR) s_hist[threadIdx.x] = 0;
    __syncthreads();
    const size_t base = (size_t)blockIdx.x * TILE_N;
    // 16-B loads (4 per thread, each wave instruction one contiguous KiB), one LDS atomic per key (one add per
    // distinct digit of each 64-key group by an 8-ballot match measured slower: C tile sort 0.137 -> 0.164 ms)
    // keys per load: 16 B of them, or 8 B (4 16-bit keys) when ITEMS is not a multiple of 8
    constexpr int KPL = ITEMS % (16 / (int)sizeof(K)) == 0 ? 16 / (int)sizeof(K) : 4;
    static_assert(ITEMS % KPL == 0, "vector key loads");
    uint32_t kv[ITEMS];
    const bool full = base + TILE_N <= n;
#pragma unroll
    for (int k = 0; k < ITEMS / KPL; ++k) {
        const size_t i = base + KPL * ((size_t)k * THREADS + threadIdx.x);
        if (full) {
            uint32_t w[4];
            if (KPL * sizeof(K) == 16) {
                const uint4 q = *reinterpret_cast<const uint4*>(keys + i);
                w[0] = q.x; w[1] = q.y; w[2] = q.z; w[3] = q.w;
            } else {
                const uint2 q = *reinterpret_cast<const uint2*>(keys + i);
                w[0] = q.x; w[1] = q.y; w[2] = w[3] = 0u;
            }
#pragma unroll
            for (int j = 0; j < KPL; ++j)
                kv[KPL * k + j] = sizeof(K) == 4 ? w[j] : (w[j >> 1] >> (16 * (j & 1))) & 0xFFFFu;
        } else {
#pragma unroll
            for (int j = 0; j < KPL; ++j) kv[KPL * k + j] = i + j < n ? (uint32_t)keys[i + j] : 0u;
        }
    }
#pragma unroll
    for (int j = 0; j < ITEMS; ++j) {
        const size_t i = base + KPL * ((size_t)(j / KPL) * THREADS + threadIdx.x) + (j % KPL);
        const bool valid = i < n;
        const uint32_t d = depth ? depth_digit(kv[j], dp.pass) : (kv[j] >> shift) & (NR - 1);
        if (valid) atomicAdd(&s_hist[d], 1u);
    }
    __syncthreads();
    if (threadIdx.x < NR) {
        if (BLOCK_MAJOR) hist[(size_t)blockIdx.x * NR + threadIdx.x] = s_hist[threadIdx.x];
        else hist[(size_t)threadIdx.x * nblocks + blockIdx.x] = s_hist[threadIdx.x];
    }
}

// One block sorts its 4096-item tile by the pass's digit in LDS, then writes each digit's run to its global
// offset (the scanned [digit][block] histogram): consecutive threads store consecutive addresses, so the scatter
// is coalesced within runs. Wave w owns the contiguous quarter [1024 w, 1024 w + 1024) of the tile and ranks its
// items in 16 rounds of 64 with wave-private running digit counts in LDS (match by 8 ballots; no block barrier
// inside the rounds); block order = (wave, round, lane) = item order, so the sort is stable.
// canon != NULL: values go to the canonical point list of the binning buffer at canon (raster_common.h).
// SELF_SCAN (small sorts, few blocks): hist is the raw block-major histogram and each block derives its global
// digit offsets itself (column prefix over the blocks before it + scan of the digit totals), which saves the
// three scan launches per pass; else hist is the scanned [digit][block] histogram.
template <typename K, bool SELF_SCAN, int ITEMS, int THREADS, bool DEPTH = false>
__global__ __launch_bounds__(THREADS) void radix_downsweep_kernel(const K* keys_in, const uint32_t* vals_in,
                                                                       K* keys_out, uint32_t* vals_out,
                                                                       size_t n_cap, const uint32_t* count, char* canon,
                                                                       int shift, const uint32_t* hist_scanned,
                                                                       uint32_t nblocks, DepthPass dp = {})
{
    constexpr int TILE_N = THREADS * ITEMS;
    constexpr int WAVES = THREADS / 64;
    constexpr int PER_WAVE = TILE_N / WAVES;
    constexpr int ROUNDS = PER_WAVE / 64;
    constexpr uint32_t NR = RADIX;
    __shared__ uint32_t s_whist[WAVES][NR];  // running digit counts per wave, then per-wave digit offsets
    __shared__ uint32_t s_dstart[NR];        // block-local start of each digit's run
    __shared__ uint32_t s_gbase[NR];         // global start of this block's run of each digit
    __shared__ uint32_t s_wave[THREADS / 64];
    __shared__ __attribute__((aligned(16))) K s_k[TILE_N];  // first the rank's peer tables (u64), when they fit
    __shared__ uint32_t s_v[TILE_N];
    constexpr bool depth = DEPTH;
    if (depth && dp.pass == DEPTH_PASSES - 1) {  // the depth sort's last pass keeps only the permutation
        keys_out = nullptr;
        vals_out = dp.vals_final;
    }
    auto digit = [&](uint32_t kk) { return depth ? depth_digit(kk, dp.pass) : (kk >> shift) & (NR - 1); };
    const size_t n = live_count(n_cap, count);
    if (canon) vals_out = reinterpret_cast<uint32_t*>(canon + canonical_list_offset(n));
    const uint32_t tid = threadIdx.x;
    const uint32_t w = tid >> 6, lane = tid & 63;
    const size_t tile0 = (size_t)blockIdx.x * TILE_N;
    static_assert(THREADS % NR == 0, "thread = digit phases");
    const bool dig = tid < NR;  // this thread also owns digit tid in the per-digit phases
    for (uint32_t i = tid; i < (uint32_t)(WAVES * NR); i += THREADS) (&s_whist[0][0])[i] = 0;
    if (SELF_SCAN) {
        uint32_t before = 0, total = 0;
        if (dig) {
            uint32_t b = 0;
            for (; b + 8 <= nblocks; b += 8) {  // 8 coalesced 1-KiB row loads in flight
                uint32_t c[8];
#pragma unroll
                for (int q = 0; q < 8; ++q) c[q] = hist_scanned[(size_t)(b + q) * NR + tid];
#pragma unroll
                for (int q = 0; q < 8; ++q) {
                    before += b + q < blockIdx.x ? c[q] : 0u;
                    total += c[q];
                }
            }
            for (; b < nblocks; ++b) {
                const uint32_t c = hist_scanned[(size_t)b * NR + tid];
                before += b < blockIdx.x ? c : 0u;
                total += c;
            }
        }
        uint32_t all;
        const uint32_t ex = block_exclusive_scan<THREADS>(total, s_wave, &all);
        if (dig) s_gbase[tid] = before + ex;
    } else if (dig) {
        s_gbase[tid] = hist_scanned[(size_t)tid * nblocks + blockIdx.x];
        // depth pass 0: block 0's start of the culled bucket = the number of visible keys, for passes 1..3
        if (depth && dp.pass == 0 && blockIdx.x == 0 && tid == DEPTH_CULLED_BUCKET) dp.words[0] = s_gbase[tid];
    }
    const size_t base = tile0 + (size_t)w * PER_WAVE + lane;
    uint32_t k[ROUNDS], v[ROUNDS], lr[ROUNDS];
#pragma unroll
    for (int r = 0; r < ROUNDS; ++r) {
        const size_t i = base + 64 * r;
        k[r] = i < n ? keys_in[i] : 0u;
        v[r] = i < n ? vals_in[i] : 0u;
    }
    __syncthreads();
    // one round's rank: LDS ops of a wave complete in issue order, so every lane reads the count before the leader's
    // add lands, and the next round's read sees it. The add needs no value back, so no round waits for the previous one
    auto rank_round = [&](int r, bool valid, uint32_t d, uint64_t peers) {
        const uint32_t rank = mask_rank(peers);
        lr[r] = (valid ? s_whist[w][d] : 0u) + rank;
        __builtin_amdgcn_wave_barrier();
        if (valid && rank == 0) atomicAdd(&s_whist[w][d], (uint32_t)__popcll(peers));
        __builtin_amdgcn_wave_barrier();
    };
#pragma unroll
    for (int r = 0; r < ROUNDS; ++r) {
        const bool valid = base + 64 * r < n;
        const uint32_t d = digit(k[r]);
        rank_round(r, valid, d, wave_match_digit<RADIX_BITS>(d, valid));
    }
    __syncthreads();
    {   // thread = digit: per-wave exclusive offsets, then the block-wide exclusive scan of the digit totals
        uint32_t run = 0;
        if (dig) {
#pragma unroll
            for (int q = 0; q < WAVES; ++q) {
                const uint32_t c = s_whist[q][tid];
                s_whist[q][tid] = run;
                run += c;
            }
        }
        uint32_t total;
        const uint32_t ex = block_exclusive_scan<THREADS>(run, s_wave, &total);
        if (dig) s_dstart[tid] = ex;
    }
    __syncthreads();
#pragma unroll
    for (int r = 0; r < ROUNDS; ++r) {
        if (base + 64 * r < n) {
            const uint32_t d = digit(k[r]);
            const uint32_t lp = s_dstart[d] + s_whist[w][d] + lr[r];
            s_k[lp] = (K)k[r];
            s_v[lp] = v[r];
        }
    }
    __syncthreads();
    const uint32_t nvalid = (uint32_t)min((size_t)TILE_N, n > tile0 ? n - tile0 : (size_t)0);
    for (uint32_t j = tid; j < nvalid; j += THREADS) {
        const uint32_t kk = s_k[j];
        const uint32_t d = digit(kk);
        const uint32_t dst = s_gbase[d] + (j - s_dstart[d]);
        if (depth && dp.pass == 0 && d == DEPTH_CULLED_BUCKET) {  // pass 0: a culled Gaussian's final place, [nvis, n) in index order
            dp.vals_final[dst] = s_v[j];
            continue;
        }
        if (!depth || keys_out) keys_out[dst] = (K)kk;  // NULL: the depth sort's last pass (only the permutation is kept)
        vals_out[dst] = s_v[j];
    }
}

// ---- single-pass ("onesweep") LSD passes with decoupled look-back ------------------------------------------
// One launch per 8-bit pass instead of upsweep + (scan) + downsweep: the digit histograms of ALL passes come from
// one read of the keys up front (onesweep_hist_kernel), and each pass block finds the global start of its digit runs
// by looking back over the blocks before it. Block v publishes, per digit, its own count (AGG) as soon as it has
// ranked its tile, then the inclusive prefix (PRE) once it knows its exclusive one; a block looking back adds AGG
// counts until it meets a PRE. Tiles are handed out by an atomic ticket, so every block a block waits on has already
// started, and no block waits on a later one: the look-back always finishes (each wait is also bounded, see below).
// The ranking inside a block is radix_downsweep_kernel's; the result is the same stable permutation.
constexpr uint32_t LB_AGG = 1u << 30, LB_PRE = 2u << 30, LB_COUNT = LB_AGG - 1u;
#ifndef OMR_LB_WINDOW
#define OMR_LB_WINDOW 8
#endif
constexpr int LB_WINDOW = OMR_LB_WINDOW;  // predecessors read per look-back round trip

// scratch words for a sort of n items over `passes` passes: status [passes][blocks][RADIX], digit totals
// [passes][RADIX], tickets [passes], error word
// keys per onesweep block: 4096, or 2048 for sorts of fewer than OS_SMALL_N keys, which then spread over more blocks
// (config B: depth sort of 100 k keys 0.059 -> 0.050 ms, tile sort of 0.35 M 0.048 -> 0.044; at config C's 1 M-key
// depth sort 2048-key tiles are slower, 0.110 vs 0.095 ms)
#ifndef OMR_OS_THREADS
#define OMR_OS_THREADS 512
#endif
constexpr int OS_THREADS = OMR_OS_THREADS;  // block size of the onesweep passes
constexpr int OS_TILE = 4096;
constexpr int OS_TILE_SMALL = 2048;
#ifndef OMR_OS_SMALL_N
#define OMR_OS_SMALL_N (1u << 19)
#endif
constexpr size_t OS_SMALL_N = OMR_OS_SMALL_N;
__host__ __device__ inline size_t os_tile(size_t n) { return n < OS_SMALL_N ? OS_TILE_SMALL : OS_TILE; }
#ifndef OMR_OS_HIST_BLOCKS
#define OMR_OS_HIST_BLOCKS 256
#endif
// histogram blocks: each digit total takes <= this many global adds (64 / 128 / 256 / 512 blocks at 1 M keys:
// 0.109 / 0.098 / 0.0945 / 0.098 ms for the whole depth sort)
constexpr uint32_t OS_HIST_BLOCKS = OMR_OS_HIST_BLOCKS;
#ifndef OMR_OS_HIST_THREADS
#define OMR_OS_HIST_THREADS 1024
#endif
constexpr int OS_HIST_THREADS = OMR_OS_HIST_THREADS;
// Onesweep only for sorts of at most this many tiles (the depth sort up to 2 M Gaussians: 0.100 vs 0.122 ms at
// 1 M). Past that the look-back chains and the same-address ticket / histogram adds cost more than the launches
// they save (the 7.9 M-instance tile sort: 0.185 vs 0.142 ms), and the upsweep / scan / downsweep passes run.
#ifndef OMR_OS_MAX_BLOCKS
#define OMR_OS_MAX_BLOCKS 512
#endif
constexpr uint32_t OS_MAX_BLOCKS = OMR_OS_MAX_BLOCKS;

__host__ __device__ inline size_t onesweep_words(size_t n, int passes)
{
    const size_t nb = (n + os_tile(n) - 1) / os_tile(n);
    return (size_t)passes * (nb * RADIX + RADIX + 1) + 1;
}

// digit totals of every pass (ghist, zeroed by the caller; OS_HIST_BLOCKS blocks, grid-stride, so every total
// takes at most OS_HIST_BLOCKS same-address global adds) and the zeroed status words of every pass
template <typename K>
__global__ __launch_bounds__(OS_HIST_THREADS) void onesweep_hist_kernel(const K* keys, size_t n_cap,
                                                                     const uint32_t* count, int first_pass, int passes,
                                                                     uint32_t* status, size_t status_words,
                                                                     uint32_t* ghist)
{
    __shared__ uint32_t s_h[4][RADIX];
    const size_t n = live_count(n_cap, count);
    const uint32_t tid = threadIdx.x;
    const size_t stride = (size_t)gridDim.x * OS_HIST_THREADS;
    for (size_t i = (size_t)blockIdx.x * OS_HIST_THREADS + tid; i < status_words; i += stride) status[i] = 0;
    for (uint32_t i = tid; i < 4u * RADIX; i += OS_HIST_THREADS) (&s_h[0][0])[i] = 0;
    __syncthreads();
    for (size_t i = (size_t)blockIdx.x * OS_HIST_THREADS + tid; i < n; i += stride) {
        const uint32_t key = keys[i];
        for (int p = 0; p < passes; ++p) atomicAdd(&s_h[p][(key >> ((first_pass + p) * RADIX_BITS)) & (RADIX - 1)], 1u);
    }
    __syncthreads();
    if (tid < RADIX)
        for (int p = 0; p < passes; ++p)
            if (s_h[p][tid]) atomicAdd(&ghist[p * RADIX + tid], s_h[p][tid]);
}

__device__ __forceinline__ void lb_store(uint32_t* p, uint32_t v)
{
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ uint32_t lb_load(const uint32_t* p)
{
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// one pass: status = this pass's [blocks][RADIX] words (zeroed), ghist = its digit totals, ticket = its tile counter;
// DEPTH: a depth-sort pass (dp: DepthPass)
template <typename K, int TILE_N, bool DEPTH = false>
__global__ __launch_bounds__(OS_THREADS) void onesweep_kernel(const K* keys_in, const uint32_t* vals_in,
                                                                K* keys_out, uint32_t* vals_out, size_t n_cap,
                                                                const uint32_t* count, char* canon, int shift,
                                                                uint32_t* status, const uint32_t* ghist,
                                                                uint32_t* ticket, uint32_t* err, DepthPass dp = {})
{
    constexpr int WAVES = OS_THREADS / 64;
    constexpr int PER_WAVE = TILE_N / WAVES;
    constexpr int ROUNDS = PER_WAVE / 64;
    constexpr uint32_t NR = RADIX;
    __shared__ uint32_t s_whist[WAVES][NR];  // running digit counts per wave, then per-wave digit offsets
    __shared__ uint32_t s_dstart[NR];        // block-local start of each digit's run
    __shared__ uint32_t s_gbase[NR];         // global start of this block's run of each digit
    __shared__ uint32_t s_wave[OS_THREADS / 64];
    __shared__ __attribute__((aligned(16))) K s_k[TILE_N];  // first the rank's peer tables (u64), when they fit
    __shared__ uint32_t s_v[TILE_N];
    __shared__ uint32_t s_vb;
    constexpr bool depth = DEPTH;
    if (depth && dp.pass == DEPTH_PASSES - 1) {  // the depth sort's last pass keeps only the permutation
        keys_out = nullptr;
        vals_out = dp.vals_final;
    }
    auto digit = [&](uint32_t kk) { return depth ? depth_digit(kk, dp.pass) : (kk >> shift) & (NR - 1); };
    const uint32_t tid = threadIdx.x;
    if (tid == 0) s_vb = atomicAdd(ticket, 1u);
    const size_t n_live = live_count(n_cap, count);
    if (canon) vals_out = reinterpret_cast<uint32_t*>(canon + canonical_list_offset(n_live));
    const uint32_t w = tid >> 6, lane = tid & 63;
    static_assert(OS_THREADS % NR == 0, "thread = digit phases");
    const bool dig = tid < NR;  // this thread also owns digit tid in the per-digit phases
    for (uint32_t i = tid; i < (uint32_t)(WAVES * NR); i += OS_THREADS) (&s_whist[0][0])[i] = 0;
    __syncthreads();
    const uint32_t vb = s_vb;
    uint32_t total;
    const uint32_t gstart = block_exclusive_scan<OS_THREADS>(dig ? ghist[tid] : 0u, s_wave, &total);
    // the depth sort's pass 0: the start of the culled bucket is the visible count (depth_sort_nvis)
    if (depth && dp.pass == 0 && dp.words && vb == 0 && tid == DEPTH_CULLED_BUCKET) dp.words[0] = gstart;
    // depth passes 1..3 sort the visible keys alone, which their digit totals count: no count word to wait for
    const size_t n = depth && dp.pass > 0 ? (size_t)total : n_live;
    const size_t tile0 = (size_t)vb * TILE_N;
    if (tile0 >= n) return;  // block-uniform; no block looks back at a tile past the live count
    const size_t base = tile0 + (size_t)w * PER_WAVE + lane;
    uint32_t k[ROUNDS], v[ROUNDS], lr[ROUNDS];
#pragma unroll
    for (int r = 0; r < ROUNDS; ++r) {
        const size_t i = base + 64 * r;
        k[r] = i < n ? keys_in[i] : 0u;
        v[r] = i < n ? vals_in[i] : 0u;
    }
    // one round's rank (in-order LDS: read, then the leader's add, as in radix_downsweep_kernel)
    auto rank_round = [&](int r, bool valid, uint32_t d, uint64_t peers) {
        const uint32_t rank = mask_rank(peers);
        lr[r] = (valid ? s_whist[w][d] : 0u) + rank;
        __builtin_amdgcn_wave_barrier();
        if (valid && rank == 0) atomicAdd(&s_whist[w][d], (uint32_t)__popcll(peers));
        __builtin_amdgcn_wave_barrier();
    };
#pragma unroll
    for (int r = 0; r < ROUNDS; ++r) {
        const bool valid = base + 64 * r < n;
        const uint32_t d = digit(k[r]);
        rank_round(r, valid, d, wave_match_digit<RADIX_BITS>(d, valid));
    }
    __syncthreads();
    {   // thread = digit: per-wave exclusive offsets, block-local digit starts, then the look-back
        uint32_t run = 0;
        if (dig) {
#pragma unroll
            for (int q = 0; q < WAVES; ++q) {
                const uint32_t c = s_whist[q][tid];
                s_whist[q][tid] = run;
                run += c;
            }
        }
        uint32_t total;
        const uint32_t ex = block_exclusive_scan<OS_THREADS>(run, s_wave, &total);
        if (dig) {
            s_dstart[tid] = ex;
            uint32_t* mine = status + (size_t)vb * NR + tid;
            uint32_t excl = 0;
            if (vb == 0) {
                lb_store(mine, LB_PRE | run);
            } else {
                lb_store(mine, LB_AGG | run);
                // look back LB_WINDOW blocks per round trip: blocks j-1, j-2, ... (nearest first) until a PRE word;
                // an unpublished word ends the window and is polled again
                uint32_t j = vb, spins = 0;
                while (true) {
                    uint32_t st[LB_WINDOW];
#pragma unroll
                    for (int q = 0; q < LB_WINDOW; ++q)
                        st[q] = j > (uint32_t)q ? lb_load(status + (size_t)(j - 1 - q) * NR + tid) : LB_PRE;
                    uint32_t used = 0;
                    bool done = false;
#pragma unroll
                    for (int q = 0; q < LB_WINDOW; ++q) {
                        if (done || used != (uint32_t)q || (st[q] & ~LB_COUNT) == 0) continue;
                        excl += st[q] & LB_COUNT;
                        ++used;
                        done = (st[q] & LB_PRE) != 0;  // block 0 always publishes PRE: j never passes it
                    }
                    if (done) break;
                    j -= used;
                    if (used == 0) {
                        if (++spins > LB_SPIN_MAX) {
                            atomicOr(err, 1u);
                            break;
                        }
                        __builtin_amdgcn_s_sleep(1);
                    }
                }
                lb_store(mine, LB_PRE | (excl + run));
            }
            s_gbase[tid] = gstart + excl;
        }
    }
    __syncthreads();
#pragma unroll
    for (int r = 0; r < ROUNDS; ++r) {
        if (base + 64 * r < n) {
            const uint32_t d = digit(k[r]);
            const uint32_t lp = s_dstart[d] + s_whist[w][d] + lr[r];
            s_k[lp] = (K)k[r];
            s_v[lp] = v[r];
        }
    }
    __syncthreads();
    const uint32_t nvalid = (uint32_t)min((size_t)TILE_N, n - tile0);
    for (uint32_t j = tid; j < nvalid; j += OS_THREADS) {
        const uint32_t kk = s_k[j];
        const uint32_t d = digit(kk);
        const uint32_t dst = s_gbase[d] + (j - s_dstart[d]);
        if (depth && dp.pass == 0 && d == DEPTH_CULLED_BUCKET) {  // pass 0: a culled Gaussian's final place, [nvis, n) in index order
            dp.vals_final[dst] = s_v[j];
            continue;
        }
        if (!depth || keys_out) keys_out[dst] = (K)kk;  // NULL: the depth sort's last pass (only the permutation is kept)
        vals_out[dst] = s_v[j];
    }
}

// the depth sort's histogram launch (onesweep path): the digit totals of all four passes from one read of the keys
// (pass 0 over every key, passes 1..3 over the visible ones) and the zeroed look-back status words of every pass
__global__ __launch_bounds__(OS_HIST_THREADS) void depth_hist_kernel(const uint32_t* keys, size_t n, uint32_t* status,
                                                                     size_t status_words, uint32_t* ghist)
{
    __shared__ uint32_t s_h[DEPTH_PASSES][RADIX];
    const uint32_t tid = threadIdx.x;
    const size_t stride = (size_t)gridDim.x * OS_HIST_THREADS;
    for (size_t i = (size_t)blockIdx.x * OS_HIST_THREADS + tid; i < status_words; i += stride) status[i] = 0;
    for (uint32_t i = tid; i < DEPTH_PASSES * RADIX; i += OS_HIST_THREADS) (&s_h[0][0])[i] = 0;
    __syncthreads();
    for (size_t i = (size_t)blockIdx.x * OS_HIST_THREADS + tid; i < n; i += stride) {
        const uint32_t key = keys[i];
        atomicAdd(&s_h[0][depth_digit(key, 0)], 1u);
        if (key != 0xFFFFFFFFu)
            for (int p = 1; p < DEPTH_PASSES; ++p) atomicAdd(&s_h[p][depth_digit(key, p)], 1u);
    }
    __syncthreads();
    if (tid < RADIX)
        for (int p = 0; p < DEPTH_PASSES; ++p)
            if (s_h[p][tid]) atomicAdd(&ghist[p * RADIX + tid], s_h[p][tid]);
}

// ---- instances -------------------------------------------------------------------------------------------
// first index r in [lo, hi) with offsets[r] > e (offsets = inclusive scan, non-decreasing)
__device__ __forceinline__ uint32_t upper_bound_u32(const uint32_t* offsets, uint32_t lo, uint32_t hi, uint32_t e)
{
    while (lo < hi) {
        const uint32_t mid = (lo + hi) >> 1;
        if (offsets[mid] > e) hi = mid;
        else lo = mid + 1;
    }
    return lo;
}

#ifndef OMR_EMIT_OWN_MAX
#define OMR_EMIT_OWN_MAX 256
#endif
constexpr uint32_t EMIT_OWN_MAX = OMR_EMIT_OWN_MAX;  // 0: every instance gathers its owner's record itself

// Emission index: block_owner[B] = the depth rank owning slot B * EMIT_SLOTS (the rank whose slot range
// [offsets[r-1], offsets[r]) contains it). One thread per rank; only ranks containing a block start write.
__global__ __launch_bounds__(256) void emit_index_kernel(HostWords hw, int P, size_t L_cap, const uint32_t* count,
                                                         const uint32_t* offsets, uint32_t* block_owner)
{
    if (hw.dst && blockIdx.x == 0 && threadIdx.x < 64) write_host_words(hw, threadIdx.x);  // the forward's count words
    const int r = blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= P || live_count(L_cap, count) == 0) return;  // block_owner holds L_cap / EMIT_SLOTS + 1 words
    const uint32_t lo = r == 0 ? 0u : offsets[r - 1], hi = offsets[r];
    for (uint32_t B = (lo + EMIT_SLOTS - 1) / EMIT_SLOTS; B * EMIT_SLOTS < hi; ++B) block_owner[B] = (uint32_t)r;
}

// instance k of a Gaussian whose rect is w tiles wide: row ky, column kx of the rect (row-major). k / w through the
// f32 reciprocal (a u32 division is ~40 VALU): for k < 2^20 the truncated quotient is off by at most one, which the
// remainder test corrects exactly
__device__ __forceinline__ void rect_slot(uint32_t k, uint32_t w, uint32_t& kx, uint32_t& ky)
{
    if (k < (1u << 20)) {
        ky = (uint32_t)((float)k * __builtin_amdgcn_rcpf((float)w));
        int rem = (int)k - (int)(ky * w);
        if (rem < 0) { --ky; rem += (int)w; }
        else if (rem >= (int)w) { ++ky; rem -= (int)w; }
        kx = (uint32_t)rem;
    } else {
        ky = k / w;
        kx = k - ky * w;
    }
}

// the tile and point-list entry of instance k of Gaussian gid (its tiles row-major over its rect)
__device__ __forceinline__ void emit_one(const float4* splat, uint32_t gid, uint32_t k, uint32_t gx, uint32_t* key,
                                         uint32_t* val)
{
    const float4* rec = splat + (size_t)gid * SPLAT_F4;  // one 64-B line: rect, position, conic + opacity
    const float4 rect = rec[3];  // {x0, y0, x1, y1} from preprocess (getRect)
    const float4 pos = rec[0], co = rec[1];
    const uint32_t x0 = __builtin_bit_cast(uint32_t, rect.x), y0 = __builtin_bit_cast(uint32_t, rect.y);
    const uint32_t w = __builtin_bit_cast(uint32_t, rect.z) - x0;
    uint32_t ky, kx;
    rect_slot(k, w, kx, ky);
    const uint32_t tx = x0 + kx, ty = y0 + ky;
    *key = ty * gx + tx;
    // the bands of the tile this instance can reach (point list entry format, raster_common.h)
    *val = gid | (band_mask<PL_BANDS>(make_float2(pos.x, pos.y), co, tx, ty, 0) << PL_GID_BITS);
}

// duplicateWithKeys (rasterizer_impl.cu:94-140) in depth order: Gaussian order[r] owns slots
// [offsets[r-1], offsets[r]) and its tiles are emitted row-major like the reference. The value carries the
// instance's band mask next to the Gaussian index (raster_common.h: point list entries). Per INSTANCE work (not per
// Gaussian as in the reference), EMIT_PER consecutive slots per thread: the stores are 16-B per lane and fully
// coalesced, a polar Gaussian spanning hundreds of tiles no longer serialises its wave, and each thread has
// EMIT_PER independent record gathers in flight (the kernel waits on memory, not on its ALU). The block's slots
// belong to ranks [block_owner[B], block_owner[B+1]]; their slot ends are staged in LDS, each thread finds the owner
// of its first slot by a binary search there and steps forward for the others.
template <typename K>
__global__ __launch_bounds__(EMIT_THREADS) void emit_kernel(int P, size_t L_cap, const uint32_t* count,
                                                            const uint32_t* order, const uint32_t* offsets,
                                                            const uint32_t* block_owner, const float4* splat,
                                                            uint32_t gx, K* tile_keys, uint32_t* gauss_vals,
                                                            char* binning)
{
    __shared__ uint32_t s_end[EMIT_SLOTS];
    __shared__ uint32_t s_start0;
    // the block's owners themselves when there are few (EMIT_OWN_MAX): their record, band-mask constants and rect
    // are gathered once per Gaussian, not once per instance
    __shared__ float4 s_own_a[EMIT_OWN_MAX > 0 ? EMIT_OWN_MAX : 1];  // x, y, t, k    | fast: x, y, k Dt, a k
    __shared__ float4 s_own_b[EMIT_OWN_MAX > 0 ? EMIT_OWN_MAX : 1];  // dd, a, x0, y0 | fast: a dd, A t, 1/A, -
    __shared__ uint4 s_own_c[EMIT_OWN_MAX > 0 ? EMIT_OWN_MAX : 1];   // x0, y0, rect width, Gaussian index
    const size_t L = live_count(L_cap, count);
    const uint32_t B = blockIdx.x;
    const size_t e0 = (size_t)B * EMIT_SLOTS;
    if (e0 >= L) return;  // block-uniform
    const uint32_t r_lo = block_owner[B];
    const uint32_t r_hi = e0 + EMIT_SLOTS < L ? block_owner[B + 1] + 1 : (uint32_t)P;  // exclusive
    const uint32_t nr = r_hi - r_lo;
    const bool staged = nr <= EMIT_SLOTS;  // block-uniform; more only with runs of empty (culled) segments
    const bool owners = nr <= EMIT_OWN_MAX;  // block-uniform
    if (staged)
        for (uint32_t i = threadIdx.x; i < nr; i += EMIT_THREADS) s_end[i] = offsets[r_lo + i];
    if (owners)
        for (uint32_t i = threadIdx.x; i < nr; i += EMIT_THREADS) {
            // an owner with an empty segment (culled: never written) is staged too and never read
            const uint32_t gid = order[r_lo + i];
            const float4* rec = splat + (size_t)gid * SPLAT_F4;
            const float4 pos = rec[0], co = rec[1], rect = rec[3];
            const BandConsts bc = band_consts(co);
            const BandSpan sp = band_span_consts(bc);
            s_own_a[i] = make_float4(pos.x, pos.y, sp.kDt, sp.ak);
            s_own_b[i] = make_float4(sp.adt, sp.At, sp.invA, 0.f);
            s_own_c[i] = make_uint4(__builtin_bit_cast(uint32_t, rect.x), __builtin_bit_cast(uint32_t, rect.y),
                                    __builtin_bit_cast(uint32_t, rect.z) - __builtin_bit_cast(uint32_t, rect.x), gid);
        }
    if (threadIdx.x == 0) s_start0 = r_lo == 0 ? 0u : offsets[r_lo - 1];
    __syncthreads();
    const size_t eb = e0 + (size_t)threadIdx.x * EMIT_PER;
    if (eb >= L) return;
    const uint32_t nmine = (uint32_t)min((size_t)EMIT_PER, L - eb);
    uint32_t rr[EMIT_PER], kk[EMIT_PER];
    if (staged) {
        uint32_t lo = 0, hi = nr;  // first i with s_end[i] > eb
        while (lo < hi) {
            const uint32_t mid = (lo + hi) >> 1;
            if (s_end[mid] > (uint32_t)eb) hi = mid;
            else lo = mid + 1;
        }
#pragma unroll
        for (int j = 0; j < EMIT_PER; ++j) {
            const uint32_t e = (uint32_t)eb + (uint32_t)j;
            if (j > 0 && (uint32_t)j < nmine)
                while (s_end[lo] <= e) ++lo;  // the last owner's end is past every slot of the block
            rr[j] = r_lo + lo;
            kk[j] = e - (lo == 0 ? s_start0 : s_end[lo - 1]);
        }
    } else {
#pragma unroll
        for (int j = 0; j < EMIT_PER; ++j) {
            const uint32_t e = (uint32_t)eb + (uint32_t)min((uint32_t)j, nmine - 1);
            const uint32_t r = upper_bound_u32(offsets, r_lo, r_hi, e);
            rr[j] = r;
            kk[j] = e - (r == 0 ? 0u : offsets[r - 1]);
        }
    }
    uint32_t key[EMIT_PER], val[EMIT_PER];
    if (owners) {
#pragma unroll
        for (int j = 0; j < EMIT_PER; ++j) {
            const uint32_t l = rr[j] - r_lo;
            const float4 oa = s_own_a[l], ob = s_own_b[l];
            const uint4 oc = s_own_c[l];
            uint32_t kx, ky;
            rect_slot(kk[j], oc.z, kx, ky);
            const uint32_t tx = oc.x + kx, ty = oc.y + ky;
            key[j] = ty * gx + tx;
            uint32_t m;
            const BandSpan sp = {oa.z, oa.w, ob.x, ob.y, ob.z};
            m = band_mask_span<PL_BANDS>(sp, make_float2(oa.x, oa.y), tx, ty);
            val[j] = oc.w | (m << PL_GID_BITS);
        }
    } else {
        uint32_t gid[EMIT_PER];
#pragma unroll
        for (int j = 0; j < EMIT_PER; ++j) gid[j] = order[rr[j]];
#pragma unroll
        for (int j = 0; j < EMIT_PER; ++j) emit_one(splat, gid[j], kk[j], gx, &key[j], &val[j]);
    }
    if (EMIT_PER % 4 == 0 && nmine == (uint32_t)EMIT_PER) {
#pragma unroll
        for (int q = 0; q < EMIT_PER; q += 4) {
            if (sizeof(K) == 4)
                *reinterpret_cast<uint4*>(tile_keys + eb + q) = make_uint4(key[q], key[q + 1], key[q + 2], key[q + 3]);
            else
                *reinterpret_cast<uint2*>(tile_keys + eb + q) =
                    make_uint2(key[q] | (key[q + 1] << 16), key[q + 2] | (key[q + 3] << 16));
            *reinterpret_cast<uint4*>(gauss_vals + eb + q) = make_uint4(val[q], val[q + 1], val[q + 2], val[q + 3]);
        }
    } else {
#pragma unroll
        for (int j = 0; j < EMIT_PER; ++j) {
            if ((uint32_t)j >= nmine) break;
            tile_keys[eb + j] = (K)key[j];
            gauss_vals[eb + j] = val[j];
        }
    }
}

// identifyTileRanges (rasterizer_impl.cu:145-167). The sorted keys of one 16-B load per thread (4 32-bit or 8 16-bit
// keys; key arrays are 16-B aligned), the predecessor of the first from the neighbouring lane.
template <typename K>
constexpr int ranges_items() { return 16 / (int)sizeof(K); }
template <typename K>
__global__ __launch_bounds__(256) void tile_ranges_kernel(size_t L_cap, const uint32_t* count, const K* tiles,
                                                          uint2* ranges)
{
    constexpr int ITEMS = ranges_items<K>();
    const size_t L = live_count(L_cap, count);
    const size_t i0 = ((size_t)blockIdx.x * blockDim.x + threadIdx.x) * ITEMS;
    if (i0 >= L) return;
    uint32_t k[ITEMS];
    if (i0 + ITEMS <= L) {
        const uint4 q = *reinterpret_cast<const uint4*>(tiles + i0);
        const uint32_t w[4] = {q.x, q.y, q.z, q.w};
#pragma unroll
        for (int j = 0; j < ITEMS; ++j) k[j] = sizeof(K) == 4 ? w[j] : (w[j >> 1] >> (16 * (j & 1))) & 0xFFFFu;
    } else {
#pragma unroll
        for (int j = 0; j < ITEMS; ++j) k[j] = i0 + j < L ? (uint32_t)tiles[i0 + j] : 0u;
    }
    uint32_t prev = i0 == 0 ? 0u : (uint32_t)tiles[i0 - 1];
#pragma unroll
    for (int j = 0; j < ITEMS; ++j) {
        const size_t idx = i0 + j;
        if (idx >= L) break;
        const uint32_t curr = k[j];
        if (idx == 0) ranges[curr].x = 0;
        else if (curr != prev) {
            ranges[prev].y = (uint32_t)idx;
            ranges[curr].x = (uint32_t)idx;
        }
        if (idx == L - 1) ranges[curr].y = (uint32_t)L;
        prev = curr;
    }
}

// Longest-first render schedule. The render kernels run one wave per tile (or half tile) and launch more waves
// than the chip holds at once; dispatching the costly tiles first keeps the SIMDs busy to the end instead of
// leaving a tail of late heavy tiles. Block c sorts the c-th of 8 contiguous shares of [0, T) — the share the
// render kernels' xcd_remap places on XCD c, so L2 locality is unchanged — by a 256-bucket counting sort on the
// cost, descending. Cost = the tile's instance count (forward) or the (instance, band) work the forward measured
// (backward). The order of equal-bucket tiles depends on LDS atomics, which is harmless: every tile is rendered
// the same way whenever it runs.
constexpr int ORDER_THREADS = 1024;
__device__ __forceinline__ uint32_t tile_cost(const uint2* ranges, const uint32_t* cost, uint32_t i)
{
    return cost ? cost[i] : ranges[i].y - ranges[i].x;
}
__global__ __launch_bounds__(ORDER_THREADS) void tile_order_kernel(const uint2* ranges, const uint32_t* cost, uint32_t T,
                                                                   uint32_t* order)
{
    __shared__ uint32_t s_hist[RADIX];
    __shared__ uint32_t s_max;
    const uint32_t lo = (uint32_t)(((uint64_t)T * blockIdx.x) / gridDim.x);
    const uint32_t hi = (uint32_t)(((uint64_t)T * (blockIdx.x + 1)) / gridDim.x);
    if (threadIdx.x < RADIX) s_hist[threadIdx.x] = 0;
    if (threadIdx.x == 0) s_max = 0;
    __syncthreads();
    uint32_t mx = 0;
    for (uint32_t i = lo + threadIdx.x; i < hi; i += ORDER_THREADS) mx = max(mx, tile_cost(ranges, cost, i));
    atomicMax(&s_max, mx);
    __syncthreads();
    const uint64_t scale = (uint64_t)s_max + 1;
    auto bucket = [&](uint32_t i) {  // 0 = costliest
        return (uint32_t)(RADIX - 1) - (uint32_t)(((uint64_t)tile_cost(ranges, cost, i) * RADIX) / scale);
    };
    for (uint32_t i = lo + threadIdx.x; i < hi; i += ORDER_THREADS) atomicAdd(&s_hist[bucket(i)], 1u);
    __syncthreads();
    {   // 256-entry exclusive scan, thread = bucket (7.5 us per launch vs 8.8 with a serial scan by one thread)
        __shared__ uint32_t s_wave[ORDER_THREADS / 64];
        const uint32_t c = threadIdx.x < RADIX ? s_hist[threadIdx.x] : 0u;
        uint32_t total;
        const uint32_t ex = block_exclusive_scan<ORDER_THREADS>(c, s_wave, &total);
        if (threadIdx.x < RADIX) s_hist[threadIdx.x] = lo + ex;
    }
    __syncthreads();
    for (uint32_t i = lo + threadIdx.x; i < hi; i += ORDER_THREADS) order[atomicAdd(&s_hist[bucket(i)], 1u)] = i;
}

// The render backward's work list (render_bwd.hip). Unit = (tile, chunk): the part of the tile's instance list in
// global chunk [chunk * CKPT, (chunk + 1) * CKPT) below the tile's last contributor. Every block scans the tiles'
// unit counts (block-wide, 1024 tiles per step), keeps the units of its own share of the list (the share xcd_remap
// maps onto XCD blockIdx.x), costs them by their positions below the tile's last contributor and counting-sorts
// them, longest first.
constexpr int SCHED_THREADS = 1024;
// tiles whose loads the schedule issues together (per-thread tile loop, share extraction)
#ifndef OMR_SCHED_UNROLL
#define OMR_SCHED_UNROLL 4
#endif
#ifndef OMR_SCHED_SG
#define OMR_SCHED_SG 8
#endif
constexpr int SCHED_LDS_UNITS = 4096;  // 48 KiB of LDS
__device__ __forceinline__ uint32_t tile_units(const uint2* ranges, const uint32_t* max_contrib, uint32_t t,
                                               uint32_t* rx, uint32_t* mc_out)
{
    uint32_t mc = 0;
#pragma unroll
    for (int g = 0; g < FWD_GROUPS; ++g) mc = max(mc, max_contrib[(size_t)t * FWD_GROUPS + g]);
    const uint2 r = ranges[t];
    mc = min(mc, r.y - r.x);
    *rx = r.x;
    *mc_out = mc;
    return mc ? (r.x + mc - 1) / CKPT - r.x / CKPT + 1 : 0u;
}
// SORTED = false (views whose units are all resident at once, render_backward_needs_order): the units go straight to
// `units` in tile order, without the costs and the counting sort.
template <bool SORTED>
__global__ __launch_bounds__(SCHED_THREADS) void backward_schedule_kernel(HostWords hw, const uint2* ranges,
                                                                          const uint32_t* max_contrib, uint32_t T,
                                                                          uint2* units_tmp, uint32_t* cost_tmp,
                                                                          uint2* units, uint32_t* unit_count)
{
    if (hw.dst && blockIdx.x == 0 && threadIdx.x < 64) write_host_words(hw, threadIdx.x);  // the backward's error word
    __shared__ uint32_t s_wave[SCHED_THREADS / 64];
    __shared__ uint32_t s_hist[RADIX];
    __shared__ uint32_t s_max;
    __shared__ uint2 s_units[SCHED_LDS_UNITS];
    __shared__ uint32_t s_cost[SCHED_LDS_UNITS];
    const uint32_t tid = threadIdx.x;
    // thread tid owns the contiguous tiles [t0, t1): one block scan of the per-thread unit counts (their loads are
    // independent, so all are in flight at once) instead of a scan per 1024 tiles — 2 x T/1024 dependent
    // load + barrier rounds cost 32 us at config C
    const uint32_t per = (T + SCHED_THREADS - 1) / SCHED_THREADS;
    const uint32_t t0 = min(T, tid * per), t1 = min(T, t0 + per);
    uint32_t mine = 0;
#pragma unroll OMR_SCHED_UNROLL
    for (uint32_t t = t0; t < t1; ++t) {
        uint32_t rx, mc;
        mine += tile_units(ranges, max_contrib, t, &rx, &mc);
    }
    uint32_t total;
    const uint32_t first0 = block_exclusive_scan<SCHED_THREADS>(mine, s_wave, &total);
    // this block's share of [0, total): xcd_remap's split over the 8 XCDs
    const uint32_t q = total / gridDim.x, rem = total % gridDim.x, x = blockIdx.x;
    const uint32_t lo = x * q + min(x, rem), hi = lo + q + (x < rem ? 1u : 0u);
    // the share's unsorted units and costs: in LDS when they fit (config C: ~3 k units per share), which saves the
    // global round trips of the three passes below; else in the global scratch
    const bool in_lds = SORTED && hi - lo <= (uint32_t)SCHED_LDS_UNITS;  // block-uniform
    uint2* uu = !SORTED ? units : in_lds ? s_units : units_tmp;
    uint32_t* cc = in_lds ? s_cost : cost_tmp;
    const uint32_t ub = in_lds ? lo : 0u;  // index of unit u = u - ub
    if (first0 < hi && first0 + mine > lo) {
        // tiles in groups of SG whose loads are all issued before the group's stores (the stores may alias the
        // loads as far as the compiler knows: one tile at a time, each load waited for a global round trip)
        constexpr uint32_t SG = OMR_SCHED_SG;
        uint32_t first = first0;
        for (uint32_t tg = t0; tg < t1 && first < hi; tg += SG) {
            uint32_t rxs[SG], mcs[SG], cs[SG];
#pragma unroll
            for (uint32_t j = 0; j < SG; ++j) cs[j] = tg + j < t1 ? tile_units(ranges, max_contrib, tg + j, &rxs[j], &mcs[j]) : 0u;
#pragma unroll
            for (uint32_t j = 0; j < SG; ++j) {
                const uint32_t t = tg + j, c = cs[j], rx = rxs[j], mc = mcs[j];
                for (uint32_t k = 0; k < c; ++k) {
                    const uint32_t u = first + k;
                    if (u < lo || u >= hi) continue;
                    const uint32_t chunk = rx / CKPT + k;
                    uu[u - ub] = make_uint2(t, chunk);
                    // cost: the segment's positions below the tile's last contributor
                    if (SORTED) cc[u - ub] = min(rx + mc, (chunk + 1) * CKPT) - max(rx, chunk * CKPT);
                }
                first += c;
            }
        }
    }
    if (!SORTED) {
        if (x == 0 && tid == 0) *unit_count = total;
        return;
    }
    if (tid < RADIX) s_hist[tid] = 0;
    if (tid == 0) s_max = 0;
    if (!in_lds) __threadfence();  // the share's entries (written by other threads of this block) before they are read back
    __syncthreads();
    uint32_t mx = 0;
    for (uint32_t u = lo + tid; u < hi; u += SCHED_THREADS) mx = max(mx, cc[u - ub]);
    atomicMax(&s_max, mx);
    __syncthreads();
    const uint64_t scale = (uint64_t)s_max + 1;
    auto bucket = [&](uint32_t u) {  // 0 = costliest
        return (uint32_t)(RADIX - 1) - (uint32_t)(((uint64_t)cc[u - ub] * RADIX) / scale);
    };
    // wave-aggregated LDS atomics: most units of a large view are full segments of one cost, so per-unit adds would
    // serialise on one bucket (config E: ~16 k per block)
    for (uint32_t u = lo + tid; u < hi; u += SCHED_THREADS) {
        const uint32_t b = bucket(u);
        const uint64_t peers = wave_match_digit<RADIX_BITS>(b, true);
        if (mask_rank(peers) == 0) atomicAdd(&s_hist[b], (uint32_t)__popcll(peers));
    }
    __syncthreads();
    {
        const uint32_t cnt = tid < RADIX ? s_hist[tid] : 0u;
        uint32_t tot;
        const uint32_t ex = block_exclusive_scan<SCHED_THREADS>(cnt, s_wave, &tot);
        if (tid < RADIX) s_hist[tid] = lo + ex;
    }
    __syncthreads();
    for (uint32_t u = lo + tid; u < hi; u += SCHED_THREADS) {  // slots per bucket, one LDS atomic per bucket and wave
        const uint32_t b = bucket(u);
        const uint64_t peers = wave_match_digit<RADIX_BITS>(b, true);
        const uint32_t rank = mask_rank(peers);
        const uint32_t leader = (uint32_t)__builtin_ctzll(peers);
        const uint32_t base0 = rank == 0 ? atomicAdd(&s_hist[b], (uint32_t)__popcll(peers)) : 0u;
        units[(uint32_t)__shfl((int)base0, (int)leader, 64) + rank] = uu[u - ub];
    }
    if (x == 0 && tid == 0) *unit_count = total;
}

}  // namespace

void launch_backward_schedule(const HostWords& hw, const uint2* ranges, const uint32_t* max_contrib, uint32_t T,
                              uint2* units_tmp, uint32_t* cost_tmp, uint2* units, uint32_t* unit_count, bool sorted,
                              hipStream_t s)
{
    if (T == 0) {
        if (hw.dst) launch_host_words(hw, s);
        return;
    }
    (sorted ? backward_schedule_kernel<true> : backward_schedule_kernel<false>)<<<8, SCHED_THREADS, 0, s>>>(
        hw, ranges, max_contrib, T, units_tmp, cost_tmp, units, unit_count);
}

__global__ void host_words_kernel(HostWords hw) { write_host_words(hw, threadIdx.x); }

void launch_host_words(const HostWords& h, hipStream_t s) { host_words_kernel<<<1, 64, 0, s>>>(h); }

void launch_tile_order(const uint2* ranges, const uint32_t* cost, uint32_t T, uint32_t* order, hipStream_t s)
{
    if (T == 0) return;
    tile_order_kernel<<<min(T, 8u), ORDER_THREADS, 0, s>>>(ranges, cost, T, order);
}

size_t scan_partials_size(size_t n) { return div_up(n, SCAN_TILE) + 1; }

size_t radix_partials_words(size_t n) { return 2 * scan_partials_size(radix_hist_size(n)) + 2; }

size_t scan2_status_words(size_t n) { return 4 * div_up(n, SCAN_TILE) + 2; }

void launch_forward_scans(const uint32_t* tiles_touched, const uint2* rects, const uint32_t* order, uint32_t* offsets,
                          uint32_t* row_first, uint32_t* row_offsets, uint2* drect, uint2* desc_r, uint32_t* huge_list,
                          uint32_t* huge_count, uint32_t* status, uint32_t* count_out, uint32_t* err, size_t n,
                          hipStream_t s, const uint32_t* nvis)
{
    if (n == 0) return;
    const uint32_t nb = div_up(n, SCAN_TILE);
    uint64_t* st = reinterpret_cast<uint64_t*>(status);  // [2][nb] 64-bit | ticket | own error word
    uint32_t* ticket = status + 4 * (size_t)nb;
    scan2_lookback_kernel<<<nb, SCAN_THREADS, 0, s>>>(tiles_touched, rects, order, n, st, st + nb, ticket,
                                                      err ? err : ticket + 1, offsets, row_first, row_offsets, drect,
                                                      reinterpret_cast<uint32_t*>(desc_r), huge_list, huge_count,
                                                      count_out, nvis);
}

size_t radix_hist_size(size_t n) { return (size_t)RADIX * div_up(n, SORT_TILE); }


static bool use_onesweep(size_t n) { return div_up(n, os_tile(n)) <= OS_MAX_BLOCKS; }

size_t radix_scratch_words(size_t n, int passes)
{
    return use_onesweep(n) ? std::max(onesweep_words(n, passes), radix_hist_size(n)) : radix_hist_size(n);
}

ZeroSpan radix_zero_span(uint32_t* hist, size_t n, int passes)
{
    ZeroSpan z;
    if (n == 0 || passes <= 0 || !use_onesweep(n)) return z;
    // digit totals [passes][RADIX] | tickets [passes] | error word, after the status words
    z.p = hist + (size_t)passes * div_up(n, os_tile(n)) * RADIX;
    z.n = (size_t)passes * (RADIX + 1) + 1;
    return z;
}

template <typename K>
int radix_sort_pairs(K* key_a, K* key_b, uint32_t* val_a, uint32_t* val_b, uint32_t* hist, uint32_t* scan_partials,
                     size_t n, const uint32_t* count, char* canon, int first_pass, int passes, hipStream_t s,
                     bool scratch_zeroed, uint32_t* err_out)
{
    if (n == 0 || passes <= 0) return 0;
    K *ki = key_a, *ko = key_b;
    uint32_t *vi = val_a, *vo = val_b;
    int cur = 0;
    if (use_onesweep(n)) {
        const uint32_t nb = div_up(n, os_tile(n));
        // scratch: status [passes][nb][RADIX] | ghist [passes][RADIX] | tickets [passes] | error word
        uint32_t* status = hist;
        uint32_t* ghist = hist + (size_t)passes * nb * RADIX;
        uint32_t* tickets = ghist + (size_t)passes * RADIX;
        uint32_t* err = err_out ? err_out : tickets + passes;
        if (!scratch_zeroed) (void)hipMemsetAsync(ghist, 0, ((size_t)passes * (RADIX + 1) + 1) * sizeof(uint32_t), s);
        onesweep_hist_kernel<K><<<std::min(div_up(n, OS_HIST_THREADS), OS_HIST_BLOCKS), OS_HIST_THREADS, 0, s>>>(
            ki, n, count, first_pass, passes, status, (size_t)passes * nb * RADIX, ghist);
        for (int p = 0; p < passes; ++p) {
            const bool last = p == passes - 1;
            auto kern = os_tile(n) == OS_TILE ? onesweep_kernel<K, OS_TILE> : onesweep_kernel<K, OS_TILE_SMALL>;
            kern<<<nb, OS_THREADS, 0, s>>>(ki, vi, ko, vo, n, count, last ? canon : nullptr,
                                            (first_pass + p) * RADIX_BITS, status + (size_t)p * nb * RADIX,
                                            ghist + (size_t)p * RADIX, tickets + p, err, DepthPass{});
            std::swap(ki, ko);
            std::swap(vi, vo);
            cur ^= 1;
        }
        return cur;
    }
    // large sorts (config E's 117 M instances) take 8192-key tiles: digit runs twice as long per block, so the
    // scattered stores fill whole lines more often (tile sort 1.98 -> 1.64 ms there); below the threshold 4096-key
    // tiles are faster (0.136 vs 0.152 ms at config C's 7.9 M)
    const bool large = n >= (sizeof(K) == 2 ? SORT_LARGE_MIN16 : SORT_LARGE_MIN);
    const uint32_t nb = div_up(n, large ? SORT_THREADS_LARGE * SORT_ITEMS_LARGE : SORT_TILE);
    for (int p = first_pass; p < first_pass + passes; ++p) {
        const int shift = p * RADIX_BITS;
        const bool last = p == first_pass + passes - 1;
        if (nb <= SELF_SCAN_MAX_BLOCKS) {
            if (large) {
                radix_upsweep_kernel<K, true, SORT_ITEMS_LARGE, SORT_THREADS_LARGE><<<nb, SORT_THREADS_LARGE, 0, s>>>(ki, n, count, shift, hist, nb,
                                                                                        nullptr, 0);
                radix_downsweep_kernel<K, true, SORT_ITEMS_LARGE, SORT_THREADS_LARGE><<<nb, SORT_THREADS_LARGE, 0, s>>>(
                    ki, vi, ko, vo, n, count, last ? canon : nullptr, shift, hist, nb);
            } else {
                radix_upsweep_kernel<K, true, SORT_ITEMS_S, SORT_THREADS_S><<<nb, SORT_THREADS_S, 0, s>>>(ki, n, count, shift, hist, nb,
                                                                                  nullptr, 0);
                radix_downsweep_kernel<K, true, SORT_ITEMS_S, SORT_THREADS_S><<<nb, SORT_THREADS_S, 0, s>>>(
                    ki, vi, ko, vo, n, count, last ? canon : nullptr, shift, hist, nb);
            }
        } else {
            // scan_partials: look-back status [nbs] (64-bit) | ticket | error word, zeroed by the upsweep
            const uint32_t nbs = div_up((size_t)RADIX * nb, SCAN_TILE);
            uint64_t* lb = reinterpret_cast<uint64_t*>(scan_partials);
            uint32_t* lb_ticket = scan_partials + 2 * (size_t)nbs;
            if (large)
                radix_upsweep_kernel<K, false, SORT_ITEMS_LARGE, SORT_THREADS_LARGE><<<nb, SORT_THREADS_LARGE, 0, s>>>(
                    ki, n, count, shift, hist, nb, scan_partials, 2 * nbs + 2);
            else
                radix_upsweep_kernel<K, false, SORT_ITEMS_S, SORT_THREADS_S><<<nb, SORT_THREADS_S, 0, s>>>(ki, n, count, shift, hist, nb,
                                                                                   scan_partials, 2 * nbs + 2);
            scan_lookback_kernel<<<std::min(nbs, SCAN_GRID_MAX), SCAN_THREADS, 0, s>>>(
                hist, hist, (size_t)RADIX * nb, nullptr, lb, lb_ticket, err_out ? err_out : lb_ticket + 1);
            if (large)
                radix_downsweep_kernel<K, false, SORT_ITEMS_LARGE, SORT_THREADS_LARGE><<<nb, SORT_THREADS_LARGE, 0, s>>>(
                    ki, vi, ko, vo, n, count, last ? canon : nullptr, shift, hist, nb);
            else
                radix_downsweep_kernel<K, false, SORT_ITEMS_S, SORT_THREADS_S><<<nb, SORT_THREADS_S, 0, s>>>(
                    ki, vi, ko, vo, n, count, last ? canon : nullptr, shift, hist, nb);
        }
        std::swap(ki, ko);
        std::swap(vi, vo);
        cur ^= 1;
    }
    return cur;
}

// ---- the depth sort (DepthPass above): four onesweep passes, or upsweep / scan / downsweep per pass -----------------
// scratch (hist): the plain sort's over four passes (radix_scratch_words), then the depth words [4]
static size_t depth_words_at(size_t n)
{
    return use_onesweep(n) ? onesweep_words(n, DEPTH_PASSES) : radix_hist_size(n);
}
size_t depth_sort_scratch_words(size_t n) { return radix_scratch_words(n, DEPTH_PASSES) + 4; }
size_t depth_sort_partials_words(size_t n) { return radix_partials_words(n); }
ZeroSpan depth_sort_zero_span(uint32_t* hist, size_t n)
{
    ZeroSpan z;
    if (n == 0) return z;
    if (use_onesweep(n)) {  // digit totals, tickets, error word (radix_zero_span), then the words, contiguous
        z = radix_zero_span(hist, n, DEPTH_PASSES);
        z.n += 4;
    } else {
        z.p = hist + depth_words_at(n);
        z.n = 4;
    }
    return z;
}

const uint32_t* depth_sort_nvis(const uint32_t* hist, size_t n) { return hist + depth_words_at(n); }

void depth_sort(uint32_t* key_a, uint32_t* key_b, uint32_t* val_a, uint32_t* val_b, uint32_t* order, uint32_t* hist,
                uint32_t* scan_partials, size_t n, hipStream_t s, uint32_t* err)
{
    if (n == 0) return;
    uint32_t* words = hist + depth_words_at(n);
    uint32_t *ki = key_a, *ko = key_b, *vi = val_a, *vo = val_b;
    if (use_onesweep(n)) {
        const uint32_t nb = div_up(n, os_tile(n));
        uint32_t* status = hist;
        uint32_t* ghist = hist + (size_t)DEPTH_PASSES * nb * RADIX;
        uint32_t* tickets = ghist + (size_t)DEPTH_PASSES * RADIX;
        depth_hist_kernel<<<std::min(div_up(n, OS_HIST_THREADS), OS_HIST_BLOCKS), OS_HIST_THREADS, 0, s>>>(
            key_a, n, status, (size_t)DEPTH_PASSES * nb * RADIX, ghist);
        for (int p = 0; p < DEPTH_PASSES; ++p) {
            DepthPass dp;
            dp.pass = p;
            dp.words = words;
            dp.vals_final = order;
            auto kern = os_tile(n) == OS_TILE ? onesweep_kernel<uint32_t, OS_TILE, true>
                                              : onesweep_kernel<uint32_t, OS_TILE_SMALL, true>;
            kern<<<nb, OS_THREADS, 0, s>>>(ki, vi, ko, vo, n, nullptr, nullptr, 0,
                                            status + (size_t)p * nb * RADIX, ghist + (size_t)p * RADIX, tickets + p,
                                            err, dp);
            std::swap(ki, ko);
            std::swap(vi, vo);
        }
        return;
    }
    const uint32_t nb = div_up(n, SORT_TILE);
    const uint32_t nbs = div_up((size_t)RADIX * nb, SCAN_TILE);
    uint64_t* lb = reinterpret_cast<uint64_t*>(scan_partials);
    uint32_t* lb_ticket = scan_partials + 2 * (size_t)nbs;
    for (int p = 0; p < DEPTH_PASSES; ++p) {
        DepthPass dp;
        dp.pass = p;
        dp.words = words;
        dp.vals_final = order;
        const uint32_t* count = p == 0 ? nullptr : words;
        radix_upsweep_kernel<uint32_t, false, SORT_ITEMS_S, SORT_THREADS_S, true><<<nb, SORT_THREADS_S, 0, s>>>(
            ki, n, count, 0, hist, nb, scan_partials, 2 * nbs + 2, dp);
        scan_lookback_kernel<<<std::min(nbs, SCAN_GRID_MAX), SCAN_THREADS, 0, s>>>(
            hist, hist, (size_t)RADIX * nb, nullptr, lb, lb_ticket, err ? err : lb_ticket + 1);
        radix_downsweep_kernel<uint32_t, false, SORT_ITEMS_S, SORT_THREADS_S, true><<<nb, SORT_THREADS_S, 0, s>>>(
            ki, vi, ko, vo, n, count, nullptr, 0, hist, nb, dp);
        std::swap(ki, ko);
        std::swap(vi, vo);
    }
}

// ---- the depth sort of small views by counting (depth_count_sort) -------------------------------------------------
// Key i lands at #{j : k_j < k_i} + #{j < i : k_j == k_i}: the stable sort's position, so the permutation is the
// radix sorts' bit for bit (ties in index order, the culled keys 0xFFFFFFFF last in index order). One launch of
// O(n^2) compares instead of a histogram and four look-back passes (config A, 10 k keys: ~30 us of chained launches).
// Workgroup = 64 keys, one per lane, x CS_WAVES waves; wave w compares them with the w-th slice of all n keys and the
// slices' counts are summed through LDS. A wave stages its slice in CS_PIECE-key pieces in its own LDS region (vector
// loads, the next piece's in flight while the current one is compared) and reads each group of 4 keys back with one
// wave-uniform ds_read_b128 (a broadcast). Each slice splits at the workgroup's own 64 keys: before them a key counts
// when <= k_i, after them when < k_i, and only the 64 in between compare indices too. At A (10 k keys, 157
// workgroups) it takes 18.8 us, bound by the compares (2 VALU each) of the 16 waves on each busy CU; reading the keys
// with wave-uniform scalar loads instead took 19.2 us (profiles/r06l_A_kernel_stats.csv, r06m_A_kernel_stats.csv).
constexpr int CS_WAVES = 16;
constexpr int CS_PIECE = 512;  // keys per wave and staged piece: 2 uint4 per lane
// keys [s, e) of a staged piece (p: its LDS words, from key index p0) that order before k_i; s, e wave-uniform
template <bool OR_EQUAL>
__device__ __forceinline__ uint32_t count_staged(const uint32_t* p, uint32_t p0, uint32_t s, uint32_t e, uint32_t ki)
{
    uint32_t c = 0, j = s;
    for (; j + 4 <= e; j += 4) {  // s - p0 is a multiple of 4 (slices, pieces and workgroups start at multiples of 4)
        const uint4 q = *reinterpret_cast<const uint4*>(p + (j - p0));
        c += OR_EQUAL ? (q.x <= ki) + (q.y <= ki) + (q.z <= ki) + (q.w <= ki)
                      : (q.x < ki) + (q.y < ki) + (q.z < ki) + (q.w < ki);
    }
    for (; j < e; ++j) c += OR_EQUAL ? (p[j - p0] <= ki) : (p[j - p0] < ki);
    return c;
}
__global__ __launch_bounds__(64 * CS_WAVES) void depth_count_sort_kernel(const uint32_t* __restrict__ keys,
                                                                         uint32_t* __restrict__ order, uint32_t n)
{
    __shared__ uint4 s_piece[CS_WAVES][CS_PIECE / 4];
    __shared__ uint32_t s_cnt[CS_WAVES][64];
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t w = (uint32_t)__builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const uint32_t b0 = blockIdx.x * 64u, i = b0 + lane, b1 = min(n, b0 + 64u);
    const uint32_t ki = i < n ? keys[i] : 0u;
    const uint32_t per = ((n + CS_WAVES - 1) / CS_WAVES + 15u) / 16u * 16u;
    const uint32_t j0 = min(n, w * per), j1 = min(n, j0 + per);
    const uint32_t* sp = reinterpret_cast<const uint32_t*>(s_piece[w]);
    static_assert(CS_PIECE == 512, "two uint4 per lane and piece");
    // lanes past the slice reload the piece's first group; a group that starts below n lies inside the keys'
    // allocation, whose end Carver rounds up to 16 B (keys past the slice are never read back)
    auto group = [&](uint32_t p0, uint32_t q) {
        const uint32_t k = p0 + 4u * (lane + 64u * q);
        return *reinterpret_cast<const uint4*>(keys + (k < j1 ? k : p0));
    };
    uint4 nx0 = make_uint4(0u, 0u, 0u, 0u), nx1 = nx0;
    if (j0 < j1) {
        nx0 = group(j0, 0);
        nx1 = group(j0, 1);
    }
    uint32_t c = 0;
    for (uint32_t p0 = j0; p0 < j1; p0 += CS_PIECE) {
        const uint32_t p1 = min(j1, p0 + CS_PIECE);
        s_piece[w][lane] = nx0;
        s_piece[w][lane + 64u] = nx1;
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");  // a wave's LDS ops complete in issue order
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        if (p1 < j1) {  // the next piece in flight while this one is compared
            nx0 = group(p1, 0);
            nx1 = group(p1, 1);
        }
        c += count_staged<true>(sp, p0, p0, min(p1, b0), ki);         // before the workgroup's keys: ties count
        c += count_staged<false>(sp, p0, max(p0, b1), p1, ki);        // after them: ties do not
        for (uint32_t j = max(p0, b0); j < min(p1, b1); ++j) {        // among them: by index
            const uint32_t kj = sp[j - p0];
            c += (kj < ki) | ((kj == ki) & (j < i));
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");  // every read of this piece before the next store
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    }
    s_cnt[w][lane] = c;
    __syncthreads();
    if (w == 0 && i < n) {
        uint32_t pos = 0;
#pragma unroll
        for (int q = 0; q < CS_WAVES; ++q) pos += s_cnt[q][lane];
        order[pos] = i;
    }
}
void depth_count_sort(const uint32_t* keys, uint32_t* order, size_t n, hipStream_t s)
{
    if (n == 0) return;
    depth_count_sort_kernel<<<div_up((uint32_t)n, 64u), 64 * CS_WAVES, 0, s>>>(keys, order, (uint32_t)n);
}

template int radix_sort_pairs<uint32_t>(uint32_t*, uint32_t*, uint32_t*, uint32_t*, uint32_t*, uint32_t*, size_t,
                                        const uint32_t*, char*, int, int, hipStream_t, bool, uint32_t*);
template int radix_sort_pairs<uint16_t>(uint16_t*, uint16_t*, uint32_t*, uint32_t*, uint32_t*, uint32_t*, size_t,
                                        const uint32_t*, char*, int, int, hipStream_t, bool, uint32_t*);

size_t emit_index_size(size_t L_cap) { return div_up(L_cap, EMIT_SLOTS) + 1; }

size_t scan_status_words(size_t n) { return 2 * (size_t)div_up(n, SCAN_TILE) + 2; }

void launch_exclusive_scan(const uint32_t* in, uint32_t* out, size_t n, const uint32_t* n_dev, uint32_t* status,
                           uint32_t* err, hipStream_t s, uint32_t mask)
{
    if (n == 0) return;
    const uint32_t nbs = div_up(n, SCAN_TILE);
    uint32_t* ticket = status + 2 * (size_t)nbs;
    scan_lookback_kernel<<<std::min(nbs, SCAN_GRID_MAX), SCAN_THREADS, 0, s>>>(
        in, out, n, n_dev, reinterpret_cast<uint64_t*>(status), ticket, err ? err : ticket + 1, mask);
}

void launch_emit_instances(const HostWords& hw, int P, size_t L_cap, const uint32_t* count, const GeomState& g,
                           uint32_t gx, uint32_t* block_owner, void* tile_keys, bool keys16, uint32_t* gauss_vals,
                           char* binning, hipStream_t s)
{
    if (P <= 0 || L_cap == 0) {
        if (hw.dst) launch_host_words(hw, s);
        return;
    }
    emit_index_kernel<<<div_up(P, 256), 256, 0, s>>>(hw, P, L_cap, count, g.offsets, block_owner);
    if (keys16)
        emit_kernel<uint16_t><<<div_up(L_cap, EMIT_SLOTS), EMIT_THREADS, 0, s>>>(
            P, L_cap, count, g.order, g.offsets, block_owner, g.splat, gx, static_cast<uint16_t*>(tile_keys), gauss_vals,
            binning);
    else
        emit_kernel<uint32_t><<<div_up(L_cap, EMIT_SLOTS), EMIT_THREADS, 0, s>>>(
            P, L_cap, count, g.order, g.offsets, block_owner, g.splat, gx, static_cast<uint32_t*>(tile_keys), gauss_vals,
            binning);
}

void launch_tile_ranges(size_t L_cap, const uint32_t* count, const void* sorted_tiles, bool keys16, uint2* ranges,
                        hipStream_t s)
{
    if (L_cap == 0) return;
    if (keys16)
        tile_ranges_kernel<<<div_up(L_cap, 256 * ranges_items<uint16_t>()), 256, 0, s>>>(
            L_cap, count, static_cast<const uint16_t*>(sorted_tiles), ranges);
    else
        tile_ranges_kernel<<<div_up(L_cap, 256 * ranges_items<uint32_t>()), 256, 0, s>>>(
            L_cap, count, static_cast<const uint32_t*>(sorted_tiles), ranges);
}

}  // namespace omr
