// bin.hip — tile binning by rows, then columns (gfx950).
//
// What it replaces: duplicateWithKeys + cub::DeviceRadixSort::SortPairs on (tile << 32 | depth) keys +
// identifyTileRanges (cuda_rasterizer/rasterizer_impl.cu:94-167, :622-679). The result is the reference's permutation
// — every Gaussian x tile instance in (tile, depth, Gaussian index) order — and the tile ranges.
//
// Why not sort instances: a Gaussian's tiles form a rect, so "which Gaussians cover tile (x, y), in depth order" splits
// into two one-dimensional questions, each answered by a stable counting pass over far fewer items than the L
// instances two radix passes move (sort.hip keeps that path for views past BIN_MAX_GRID tiles a side):
//   rows pass    items = the visible Gaussians in depth order, each covering the tile rows [y0, y1) of its rect. The
//                forward scans (launch_forward_scans) already give the depth-ordered rect words, the row slots (M =
//                sum of rect heights: 2.35 M at config C against 7.9 M instances, 18.4 M against 117 M at E) and each
//                2048-slot chunk's owner ranks. Output: the row entries — for every tile row, the Gaussians covering
//                it, in depth order, each with its rect width, x0 and first instance slot (the columns pass's slot
//                numbering: row-major, depth order within a row).
//   columns pass items = the row entries, each covering the columns [x0, x1) of its row. Output: the point list —
//                for every tile, its Gaussians in depth order — and the tile ranges, from the counts alone.
// Each pass cuts its expanded slots into chunks of 2048 (the columns pass never lets a chunk straddle a row, so a
// chunk's digits are the columns of one row) and runs as hist -> scan -> scatter:
//   hist     per chunk, the per-bucket counts from the owners' slot ranges: two LDS adds per owner into a
//            difference array, not one per slot (the rows pass also sums the entries' widths per row);
//   scan     one persistent decoupled-look-back launch over the [bucket][chunk] counts (sort.hip:
//            launch_exclusive_scan);
//   scatter  per chunk, every slot finds its owner in an LDS owner map (owners marked at their first slot, filled by a
//            max-scan), is ranked by its bucket inside the block (wave64 match by ballots, as the radix downsweep ranks
//            digits; wave-private running counts, so the rank keeps slot order), sorted in LDS and written as runs to
//            (scanned count + rank).
// Stable in both passes, so the point list equals the reference's bit for bit (tests/test_gpu_parity.py). The point
// list entries carry the band masks (raster_common.h), from the per-Gaussian constants preprocess stores in bin_rec;
// the columns scatter loads the next chunk's owners and constants into registers while it ranks the current one.
// The chunk descriptors need no search: the rows pass's come from the forward scans, the columns pass's from the row
// entries that hold a chunk's first slot (rows_scatter_kernel). Ranges need no key array: tile t's range is the
// scanned count at its first chunk and at the next tile's.
#include <algorithm>

#include <cstdlib>

#include "kernels.h"

namespace omr {

namespace {

// chunk geometry: THREADS threads, ITEMS slots each; slots are laid out in rounds (slot = wave * PER_WAVE + 64 r +
// lane), so a round of a wave is 64 consecutive slots
template <int THREADS_, int ITEMS_>
struct Geo {
    static constexpr int THREADS = THREADS_, ITEMS = ITEMS_, WAVES = THREADS / 64;
    static constexpr uint32_t N = (uint32_t)THREADS * ITEMS;
    static constexpr int PER_WAVE = (int)N / WAVES, ROUNDS = PER_WAVE / 64;
};
using RowGeo = Geo<256, 8>;  // rows pass: 2048-slot chunks
// columns pass: 2048-slot chunks, 1024 for small views, 4096 for large views (BinArgs::cb_shift; 4096: half the
// chunks, fewer counts to scan and fewer descriptors and barriers per instance, at the same 16 waves per CU — config E
// tile sort 1.27 -> 1.17 ms, while config C, whose 2048-slot chunks are only ~7 per block, lost 7 us to the coarser
// tail)
using ColGeoS = Geo<256, 8>;
using ColGeoL = Geo<512, 8>;
// small views: 512- or 1024-slot chunks on one- or two-wave blocks, so a few thousand instances still spread over
// many CUs (config A: 22 k instances were 11 chunks of 2048, 11 blocks on 256 CUs)
using ColGeoT = Geo<64, 8>;
using ColGeoM = Geo<128, 8>;
constexpr int RB_THREADS = RowGeo::THREADS;
constexpr int RB_ITEMS = RowGeo::ITEMS;
constexpr uint32_t RB_N = RowGeo::N;  // slots per rows-pass chunk
static_assert(RB_N == BIN_CHUNK, "launch_forward_scans cuts the rows pass's chunks at BIN_CHUNK slots");
constexpr int RB_WAVES = RowGeo::WAVES;
constexpr int RB_PER_WAVE = RowGeo::PER_WAVE;
constexpr int RB_ROUNDS = RowGeo::ROUNDS;
static_assert(ColGeoT::N == 1u << 9 && ColGeoM::N == 1u << 10 && ColGeoS::N == 1u << 11 && ColGeoL::N == 1u << 12,
              "cb_shift 9 .. 12");
// grid caps of the grid-stride chunk kernels (256 CUs: 8 resident hist blocks of 256 threads, 4 scatter blocks of
// 256 threads and <= 40 KiB LDS, or 2 of 512 threads and <= 80 KiB)
constexpr uint32_t BIN_GRID_HIST = 2048, BIN_GRID_SCATTER = 1024;
// Every rows_scatter block derives the per-row info itself (a scan over the rows) and block 0 publishes what the
// columns pass reads, instead of a one-block rows_info launch between them. The rows and columns scatters rank by LDS
// OR peer tables (rank_items) where the digit has 8 bits, by ballot matches otherwise. (The launch-separated info and
// the all-ballot ranks measured slower, §4; their code is in profiles/r04_pruned_experiments.patch.)

#ifdef OMR_BIN_STAMPS  // diagnostic: per-phase s_memrealtime stamps of cols_scatter_kernel (profiles/bin_stamps.py)
constexpr int BSTAMP_ITERS = 16, BSTAMP_PH = 8;
__device__ uint64_t g_bin_stamps[BIN_GRID_SCATTER * 4][BSTAMP_ITERS][BSTAMP_PH];  // the one-wave chunks' grid
#define BSTAMP(it, ph)                                                                             \
    do {                                                                                           \
        const uint64_t t_ = __builtin_amdgcn_s_memrealtime();                                      \
        if (threadIdx.x == 0 && (it) < (uint32_t)BSTAMP_ITERS) g_bin_stamps[blockIdx.x][it][ph] = t_; \
    } while (0)
#else
#define BSTAMP(it, ph) \
    do {               \
    } while (0)
#endif

__device__ __forceinline__ uint32_t live_L(const uint32_t* counters, size_t cap)
{
    return (uint32_t)binning_count(counters, cap);
}
__device__ __forceinline__ uint32_t live_M(const uint32_t* counters, size_t cap)
{
    return binning_count(counters, cap) ? counters[4] : 0u;
}

// Chunk order of the grid-stride kernels: the dispatcher deals blocks to the 8 XCDs round-robin (block b on XCD
// b % 8), so XCD x takes the x-th eighth of the chunks and its blocks stride over that range: blocks running together
// on one XCD work on neighbouring chunks, whose count words and point-list runs share cache lines in that XCD's L2
// (rather than partial lines written back from eight L2s). Grids that are not a multiple of 8 stride plainly.
struct ChunkRange {
    uint32_t first, end, step;
};
__device__ __forceinline__ ChunkRange xcd_chunks(uint32_t C)
{
    const uint32_t G = gridDim.x, b = blockIdx.x;
    if (G % 8u != 0u) return {b, C, G};
    const uint32_t x = b % 8u;
    return {(uint32_t)((uint64_t)C * x / 8u) + b / 8u, (uint32_t)((uint64_t)C * (x + 1u) / 8u), G / 8u};
}

// block-wide exclusive scan (THREADS threads, one value each)
template <int THREADS>
__device__ __forceinline__ uint32_t bin_block_scan(uint32_t x, uint32_t* s_wave, uint32_t* total)
{
    const uint32_t lane = threadIdx.x & 63u, w = threadIdx.x >> 6;
    const uint32_t inc = wave_incl_sum_u32(x);
    if (lane == 63) s_wave[w] = inc;
    __syncthreads();
    uint32_t off = 0, tot = 0;
#pragma unroll
    for (int k = 0; k < THREADS / 64; ++k) {
        const uint32_t v = s_wave[k];
        if ((uint32_t)k < w) off += v;
        tot += v;
    }
    __syncthreads();
    *total = tot;
    return off + inc - x;
}

// counts of `nbuckets` buckets from the difference array s_diff[0..nbuckets] (in place: s_diff[b] = count of b),
// block of THREADS threads; nbuckets <= THREADS * 4
template <int THREADS>
__device__ __forceinline__ void diff_to_counts(int* s_diff, uint32_t nbuckets, uint32_t* s_wave)
{
    constexpr int PER = 4;
    int v[PER];
    int sum = 0;
#pragma unroll
    for (int q = 0; q < PER; ++q) {
        const uint32_t b = threadIdx.x * PER + q;
        v[q] = b < nbuckets ? s_diff[b] : 0;
        sum += v[q];
    }
    uint32_t tot;
    int run = (int)bin_block_scan<THREADS>((uint32_t)sum, s_wave, &tot);
#pragma unroll
    for (int q = 0; q < PER; ++q) {
        const uint32_t b = threadIdx.x * PER + q;
        run += v[q];
        if (b < nbuckets) s_diff[b] = run;  // inclusive prefix of the differences = the count
    }
    __syncthreads();
}

// Owner of every slot of a chunk, s_own[j] = the owner holding slot s0 + j: the caller zeroes s_own, marks each owner
// at its first slot in the chunk (owners have distinct first slots; the first owner, which may start before s0, is 0),
// and this fills the runs by an inclusive max-scan — one LDS read per slot afterwards instead of walking owner ends.
template <class G>
__device__ __forceinline__ void owner_fill(uint16_t* s_own, uint32_t* s_wave)
{
    static_assert(G::ITEMS == 8, "one 16-byte LDS word of 8 owners per thread");
    const uint32_t lane = threadIdx.x & 63u, w = threadIdx.x >> 6;
    uint4 q = reinterpret_cast<const uint4*>(s_own)[threadIdx.x];
    uint32_t v[8] = {q.x & 0xFFFFu, q.x >> 16, q.y & 0xFFFFu, q.y >> 16, q.z & 0xFFFFu, q.z >> 16, q.w & 0xFFFFu, q.w >> 16};
#pragma unroll
    for (int i = 1; i < 8; ++i) v[i] = max(v[i], v[i - 1]);
    const uint32_t inc = wave_incl_max_u32(v[7]);
    if (lane == 63) s_wave[w] = inc;
    uint32_t prev = (uint32_t)__shfl_up((int)inc, 1, 64);
    if (lane == 0) prev = 0;
    __syncthreads();
#pragma unroll
    for (int k = 0; k < G::WAVES; ++k)
        if ((uint32_t)k < w) prev = max(prev, s_wave[k]);
#pragma unroll
    for (int i = 0; i < 8; ++i) v[i] = max(v[i], prev);
    reinterpret_cast<uint4*>(s_own)[threadIdx.x] =
        make_uint4(v[0] | v[1] << 16, v[2] | v[3] << 16, v[4] | v[5] << 16, v[6] | v[7] << 16);
    __syncthreads();
}

// Ranks G::ITEMS items per lane in round layout (item = wave * PER_WAVE + 64 r + lane, i.e. slot order) by digit
// d[r] < 2^BITS, stably: on return lp[r] = the item's position in the block's digit-sorted order and s_dstart[d] =
// the block-local start of digit d. s_whist: [WAVES][2^BITS] scratch. Matches radix_downsweep_kernel (sort.hip).
// s_peer_all (optional, [WAVES][2^BITS] u64, free from the first barrier on): the rounds' peer masks by LDS ORs
// instead of ballot matches.
template <int BITS, class G>
__device__ __forceinline__ void rank_items(const uint32_t (&d)[G::ROUNDS], const bool (&valid)[G::ROUNDS],
                                           uint32_t (&lp)[G::ROUNDS], uint32_t (*s_whist)[1 << BITS],
                                           uint32_t* s_dstart, uint32_t* s_wave, uint64_t* s_peer_all = nullptr)
{
    constexpr uint32_t NB = 1u << BITS;
    const uint32_t tid = threadIdx.x, w = tid >> 6;
    for (uint32_t i = tid; i < G::WAVES * NB; i += G::THREADS) (&s_whist[0][0])[i] = 0;
    __syncthreads();
    // per round: the lanes with this lane's digit (a match by BITS ballots); the group's lowest lane advances the wave's
    // running count of the digit after every lane of the wave has read it, with an add that returns nothing (a
    // ds_add_rtn per group plus a broadcast measured slower: config E tile sort 1.78 vs 2.14 ms)
    uint32_t lr[G::ROUNDS];
    uint64_t pm[G::ROUNDS];
    if (s_peer_all) {  // peer masks by LDS ORs (raster_common.h), the tables overlaid on storage free from here on
        wave_peer_masks<G::ROUNDS, NB>(d, valid, pm, s_peer_all + (size_t)w * NB);
    } else {
#pragma unroll
        for (int r = 0; r < G::ROUNDS; ++r) pm[r] = wave_match_digit<BITS>(d[r], valid[r]);
    }
#pragma unroll
    for (int r = 0; r < G::ROUNDS; ++r) {
        const uint64_t peers = pm[r];
        const uint32_t rank = mask_rank(peers);
        // LDS ops of a wave complete in issue order: every lane reads the count before the leader's add lands, and
        // the next round's read sees it; the add returns nothing, so no round waits for the previous one's read
        lr[r] = (valid[r] ? s_whist[w][d[r]] : 0u) + rank;
        __builtin_amdgcn_wave_barrier();
        if (valid[r] && rank == 0) atomicAdd(&s_whist[w][d[r]], (uint32_t)__popcll(peers));
        __builtin_amdgcn_wave_barrier();
    }
    __syncthreads();
    // per digit: per-wave exclusive offsets, then the block-wide exclusive scan of the digit totals
    constexpr uint32_t DPT = (NB + G::THREADS - 1) / G::THREADS;  // digits per thread
    uint32_t run[DPT], tsum = 0;
#pragma unroll
    for (uint32_t q = 0; q < DPT; ++q) {
        const uint32_t dg = tid * DPT + q;
        run[q] = 0;
        if (dg < NB) {
#pragma unroll
            for (int ww = 0; ww < G::WAVES; ++ww) {
                const uint32_t c = s_whist[ww][dg];
                s_whist[ww][dg] = run[q];
                run[q] += c;
            }
        }
        tsum += run[q];
    }
    uint32_t total;
    uint32_t ex = bin_block_scan<G::THREADS>(tsum, s_wave, &total);
#pragma unroll
    for (uint32_t q = 0; q < DPT; ++q) {
        const uint32_t dg = tid * DPT + q;
        if (dg < NB) s_dstart[dg] = ex;
        ex += run[q];
    }
    __syncthreads();
#pragma unroll
    for (int r = 0; r < G::ROUNDS; ++r) lp[r] = valid[r] ? s_dstart[d[r]] + s_whist[w][d[r]] + lr[r] : 0u;
}

// ---- rows pass -------------------------------------------------------------------------------------------------
// chunk c = row slots [c N, c N + N) of the M slots (depth rank r owns [row_off[r-1], row_off[r]): its rect rows);
// live chunks: div_up(M, N), their owners in desc_r (launch_forward_scans). hist_r is [2][row][live chunk]: the entry
// counts, then the sums of the entries' rect widths (scanned together: the second half's prefixes come out offset by
// M, the first half's total).
__device__ __forceinline__ uint32_t row_chunks(uint32_t M) { return (M + RB_N - 1) / RB_N; }

struct RowChunk {
    uint32_t s0, s1, r_lo, nr;  // slots; owners r_lo .. r_lo + nr - 1
};
__device__ __forceinline__ RowChunk row_chunk(const BinArgs& a, uint32_t c, uint32_t M)
{
    const uint2 d = a.desc_r[c];
    RowChunk k;
    k.s0 = c * RB_N;
    k.s1 = min(M, k.s0 + RB_N);
    k.r_lo = d.x;
    k.nr = d.y - d.x + 1u;
    return k;
}
// rect word (preprocess): rows | y0 << 11 | width << 21, x0
__device__ __forceinline__ uint32_t rect_y0(uint2 rw) { return (rw.x >> RECT_ROWS_BITS) & 0x3FFu; }
__device__ __forceinline__ uint32_t rect_w(uint2 rw) { return rw.x >> 21; }

// The binning's first kernel (grid-stride over the row chunks): zeroes the look-back words of the two scans, writes
// the forward's host words and the live lengths, and per chunk the entry counts and width sums per tile row from two
// difference arrays (two LDS adds each per owner, not one per slot). Owners are read in depth order (drect,
// row_offsets): no gathers.
__global__ __launch_bounds__(RB_THREADS) void rows_hist_kernel(BinArgs a)
{
    __shared__ int s_cnt[BIN_MAX_GRID + 1], s_wsum[BIN_MAX_GRID + 1];
    __shared__ uint32_t s_wave[RB_WAVES];
    const uint32_t tid = threadIdx.x;
    {
        const size_t gt = (size_t)blockIdx.x * RB_THREADS + tid, nt = (size_t)gridDim.x * RB_THREADS;
        for (size_t i = gt; i < a.nzero; i += nt) a.zero[i] = 0u;
    }
    if (blockIdx.x == 0 && tid < 64 && a.hw.dst) write_host_words(a.hw, tid);  // the forward's count words (capi.hip)
    const uint32_t M = live_M(a.counters, a.cap), C = row_chunks(M), gy = a.gy;
    if (blockIdx.x == 0 && tid == 0) {
        a.words[0] = M;
        a.words[2] = 2u * gy * C;
    }
    const size_t half = (size_t)gy * C;
    const ChunkRange cr = xcd_chunks(C);
    for (uint32_t c = cr.first; c < cr.end; c += cr.step) {
        for (uint32_t y = tid; y <= gy; y += RB_THREADS) {
            s_cnt[y] = 0;
            s_wsum[y] = 0;
        }
        const RowChunk k = row_chunk(a, c, M);
        __syncthreads();
        for (uint32_t i = tid; i < k.nr; i += RB_THREADS) {
            const uint32_t r = k.r_lo + i;
            const uint32_t end = a.row_offsets[r];
            const uint2 rw = a.drect[r];
            const uint32_t start = end - (rw.x & ((1u << RECT_ROWS_BITS) - 1u));
            const uint32_t ja = max(k.s0, start) - start, jb = min(k.s1, end) - start;
            const uint32_t y0 = rect_y0(rw);
            const int wd = (int)rect_w(rw);
            atomicAdd(&s_cnt[y0 + ja], 1);
            atomicAdd(&s_cnt[y0 + jb], -1);
            atomicAdd(&s_wsum[y0 + ja], wd);
            atomicAdd(&s_wsum[y0 + jb], -wd);
        }
        __syncthreads();
        diff_to_counts<RB_THREADS>(s_cnt, gy, s_wave);
        diff_to_counts<RB_THREADS>(s_wsum, gy, s_wave);
        for (uint32_t y = tid; y < gy; y += RB_THREADS) {
            a.hist_r[(size_t)y * C + c] = (uint32_t)s_cnt[y];
            a.hist_r[half + (size_t)y * C + c] = (uint32_t)s_wsum[y];
        }
        __syncthreads();
    }
}

// ---- between the scans -------------------------------------------------------------------------------------------
// Run by every rows_scatter block: per row y, its first entry and first instance slot (the scanned counts and width
// sums at chunk 0), chunk count and first chunk of the columns pass: ri[y] = {entry, slot, chunk_base, chunks} for rows
// [0, gy] (gy: the terminator), in LDS; THREADS threads, NRI rows per thread. `publish` (block 0): also the live lengths
// of the columns pass, the zero past its counts that the scan turns into their total (the last tile's end), and the
// owner end of every row's last columns chunk (rows_scatter_kernel writes the other owner words of desc_b).
template <int THREADS, int NRI>
__device__ __forceinline__ void rows_info(const BinArgs& a, uint4* ri, bool publish, uint32_t* s_wave)
{
    const uint32_t gy = a.gy, tid = threadIdx.x;
    const uint32_t L = live_L(a.counters, a.cap), M = live_M(a.counters, a.cap), C = row_chunks(M);
    const size_t half = (size_t)gy * C;
    auto entry = [&](uint32_t yy) { return yy < gy ? a.hist_r[(size_t)yy * C] : M; };
    auto slot = [&](uint32_t yy) { return yy < gy ? a.hist_r[half + (size_t)yy * C] - M : L; };
    uint32_t e0[NRI], sl0[NRI], n[NRI], tsum = 0;
#pragma unroll
    for (int q = 0; q < NRI; ++q) {
        const uint32_t y = tid * NRI + q;
        e0[q] = sl0[q] = n[q] = 0;
        if (y < gy && L) {
            e0[q] = entry(y);
            sl0[q] = slot(y);
            n[q] = (slot(y + 1) - sl0[q] + (1u << a.cb_shift) - 1u) >> a.cb_shift;
        }
        tsum += n[q];
    }
    uint32_t total;
    uint32_t cb = bin_block_scan<THREADS>(tsum, s_wave, &total);
#pragma unroll
    for (int q = 0; q < NRI; ++q) {
        const uint32_t y = tid * NRI + q;
        if (y < gy) {
            ri[y] = make_uint4(e0[q], sl0[q], cb, n[q]);
            if (publish && n[q]) reinterpret_cast<uint32_t*>(a.desc_b)[8 * (size_t)(cb + n[q] - 1) + 7] = entry(y + 1);
        }
        cb += n[q];
    }
    if (tid == 0) {
        ri[gy] = make_uint4(M, L, total, 0u);
        if (publish) {
            a.words[1] = total;
            a.words[3] = total * a.gx + 1u;
            a.hist_b[(size_t)total * a.gx] = 0u;
        }
    }
}

// Per chunk: expand the slots to (owner, row), rank them by row, write the row entries (Gaussian, width | x0 << 16)
// and their first instance slots: the row's width prefix at this chunk (the scanned width sums) plus the widths of the
// row's earlier entries in the chunk (a block scan over the row-sorted slots) — the columns pass's slot numbering,
// row-major, in depth order within a row. An entry whose instances hold a columns chunk's first slot writes that
// chunk's descriptor (and the owner end of the chunk before it): desc_b, no search.
template <int BITS>
__global__ __launch_bounds__(RB_THREADS) void rows_scatter_kernel(BinArgs a)
{
    // phase 1 (expansion): per owner, its first row minus its first slot (slot s is row s + s_yoff); phase 2
    // (write-out): the slots sorted by row, owner | row << 16
    __shared__ __attribute__((aligned(16))) uint32_t s_yoff_sorted[RB_N];  // also the rank's peer tables (u64)
    __shared__ uint32_t s_gid[RB_N];
    __shared__ uint32_t s_xw[RB_N];  // the entry word: rect width | x0 << 16
    __shared__ __attribute__((aligned(16))) uint16_t s_own[RB_N];
    __shared__ uint32_t s_whist[RB_WAVES][1 << BITS];  // | phase 2: the width prefix at each row's first sorted slot
    __shared__ uint32_t s_dstart[1 << BITS];
    __shared__ uint32_t s_gbase[1 << BITS];
    __shared__ uint32_t s_wbase[1 << BITS];
    __shared__ uint32_t s_wave[RB_WAVES];
    __shared__ uint32_t s_qtot[RB_ITEMS][RB_WAVES];
    static_assert(BITS != 8 || sizeof(s_yoff_sorted) >= RB_WAVES * 256 * sizeof(uint64_t), "peer tables fit s_yoff");
    const uint32_t tid = threadIdx.x, lane = tid & 63u, w = tid >> 6;
    const uint32_t M = live_M(a.counters, a.cap), C = row_chunks(M), gy = a.gy;
    const size_t half = (size_t)gy * C;
    uint32_t* desc_w = reinterpret_cast<uint32_t*>(a.desc_b);
    const uint32_t cbn = 1u << a.cb_shift;  // columns-pass chunk size
    // software pipeline: the next chunk's owners (first RP x 256) and count bases are loaded into registers while the
    // current chunk is ranked and written
    constexpr int RP = 3, GBP = (1 << BITS) / RB_THREADS;
    uint32_t p_end[RP], p_rx[RP], p_ry[RP], p_gid[RP], p_gb[GBP], p_wb[GBP];
    auto load_owners = [&](const RowChunk& q, uint32_t cq) {
#pragma unroll
        for (int j = 0; j < RP; ++j) {
            const uint32_t i = tid + j * RB_THREADS;
            if (i < q.nr) {
                const uint32_t r = q.r_lo + i;
                p_end[j] = a.row_offsets[r];
                const uint2 rw = a.drect[r];
                p_rx[j] = rw.x;
                p_ry[j] = rw.y;
                p_gid[j] = a.order[r];
            }
        }
#pragma unroll
        for (int j = 0; j < GBP; ++j) {
            const uint32_t y = tid + j * RB_THREADS;
            if (y < gy) {
                p_gb[j] = a.hist_r[(size_t)y * C + cq];
                p_wb[j] = a.hist_r[half + (size_t)y * C + cq];
            }
        }
    };
    __shared__ uint4 s_ri[(1 << BITS) + 1];
    rows_info<RB_THREADS, (1 << BITS) / RB_THREADS>(a, s_ri, blockIdx.x == 0, s_wave);
    __syncthreads();
    const uint4* rowinfo = s_ri;
    const ChunkRange cr = xcd_chunks(C);
    if (C == 0) return;  // nothing binned (L = 0, a capacity overflow, a failed look-back): desc_r has no entry
    RowChunk k = row_chunk(a, min(cr.first, C - 1u), M);
    if (cr.first < cr.end) load_owners(k, cr.first);
    for (uint32_t c = cr.first; c < cr.end; c += cr.step) {
        const uint32_t cn = c + cr.step;
        const RowChunk kn = row_chunk(a, min(cn, C - 1u), M);
        uint32_t* s_yoff = s_yoff_sorted;
        reinterpret_cast<uint4*>(s_own)[tid] = make_uint4(0u, 0u, 0u, 0u);
        __syncthreads();
        auto stage = [&](uint32_t i, uint32_t end, uint32_t rx, uint32_t ry, uint32_t gid) {
            const uint32_t start = end - (rx & ((1u << RECT_ROWS_BITS) - 1u));
            s_yoff[i] = rect_y0(make_uint2(rx, ry)) - start;  // modular: s + (y0 - start) = y0 + (s - start)
            s_gid[i] = gid;
            s_xw[i] = rect_w(make_uint2(rx, ry)) | (ry << 16);
            if (start >= k.s0 && start < end) s_own[start - k.s0] = (uint16_t)i;
        };
#pragma unroll
        for (int j = 0; j < RP; ++j)
            if (tid + j * RB_THREADS < k.nr) stage(tid + j * RB_THREADS, p_end[j], p_rx[j], p_ry[j], p_gid[j]);
        for (uint32_t i = tid + RP * RB_THREADS; i < k.nr; i += RB_THREADS) {
            const uint32_t r = k.r_lo + i;
            const uint2 rw = a.drect[r];
            stage(i, a.row_offsets[r], rw.x, rw.y, a.order[r]);
        }
#pragma unroll
        for (int j = 0; j < GBP; ++j) {
            const uint32_t y = tid + j * RB_THREADS;
            if (y < gy) {
                s_gbase[y] = p_gb[j];
                s_wbase[y] = p_wb[j] - M;
            }
        }
        __syncthreads();
        if (cn < cr.end) load_owners(kn, cn);
        owner_fill<RowGeo>(s_own, s_wave);
        uint32_t d[RB_ROUNDS], own[RB_ROUNDS], lp[RB_ROUNDS];
        bool valid[RB_ROUNDS];
#pragma unroll
        for (int r = 0; r < RB_ROUNDS; ++r) {
            const uint32_t j = w * RB_PER_WAVE + 64u * r + lane, s = k.s0 + j;
            valid[r] = s < k.s1;
            const uint32_t o = s_own[j];
            d[r] = valid[r] ? s + s_yoff[o] : 0u;
            own[r] = o;
        }
        // its barriers end the expansion's reads of s_yoff, whose storage then holds the peer tables
        rank_items<BITS, RowGeo>(d, valid, lp, s_whist, s_dstart, s_wave,
                                 BITS == 8 ? reinterpret_cast<uint64_t*>(s_yoff_sorted) : nullptr);
        uint32_t* s_sorted = s_yoff_sorted;
#pragma unroll
        for (int r = 0; r < RB_ROUNDS; ++r)
            if (valid[r]) s_sorted[lp[r]] = own[r] | (d[r] << 16);
        __syncthreads();
        // the width prefix over the row-sorted chunk (round layout: sorted slot j = 256 q + tid), then per row from the
        // row's first sorted slot
        const uint32_t nvalid = k.s1 - k.s0;
        uint32_t e8[RB_ITEMS], wp[RB_ITEMS];
#pragma unroll
        for (int q = 0; q < RB_ITEMS; ++q) {
            const uint32_t j = q * RB_THREADS + tid;
            e8[q] = j < nvalid ? s_sorted[j] : 0u;
            const uint32_t wd = j < nvalid ? (s_xw[e8[q] & 0xFFFFu] & 0xFFFFu) : 0u;
            const uint32_t inc = wave_incl_sum_u32(wd);
            wp[q] = inc - wd;  // exclusive within the wave
            if (lane == 63) s_qtot[q][w] = inc;
        }
        __syncthreads();
        {
            uint32_t run = 0;  // the totals of every (round, wave) before this thread's, in slot order
#pragma unroll
            for (int q = 0; q < RB_ITEMS; ++q) {
                uint32_t before = 0, all = 0;
#pragma unroll
                for (int ww = 0; ww < RB_WAVES; ++ww) {
                    const uint32_t t = s_qtot[q][ww];
                    before += (uint32_t)ww < w ? t : 0u;
                    all += t;
                }
                wp[q] += run + before;
                run += all;
            }
        }
        uint32_t* s_rowp = &s_whist[0][0];  // rank_items is done with it
#pragma unroll
        for (int q = 0; q < RB_ITEMS; ++q) {
            const uint32_t j = q * RB_THREADS + tid;
            const uint32_t y = e8[q] >> 16;
            if (j < nvalid && j == s_dstart[y]) s_rowp[y] = wp[q];
        }
        __syncthreads();
#pragma unroll
        for (int q = 0; q < RB_ITEMS; ++q) {
            const uint32_t j = q * RB_THREADS + tid;
            if (j >= nvalid) continue;
            const uint32_t oi = e8[q] & 0xFFFFu, y = e8[q] >> 16;
            const uint32_t dst = s_gbase[y] + (j - s_dstart[y]);
            const uint32_t xw = s_xw[oi], ex = s_wbase[y] + (wp[q] - s_rowp[y]);
            a.ent_gid[dst] = s_gid[oi];
            a.ent_w[dst] = xw;
            a.ent_ex[dst] = ex;
            // the columns chunk whose first slot this entry holds (widths <= BIN_MAX_GRID < 2048: at most one)
            const uint4 ri = rowinfo[y];
            const uint32_t rel = ex - ri.y, kk = (rel + cbn - 1u) >> a.cb_shift;
            if (kk < ri.w && (kk << a.cb_shift) < rel + (xw & 0xFFFFu)) {
                const uint32_t cc = ri.z + kk, s0 = ri.y + (kk << a.cb_shift);
                const uint32_t s1 = min(rowinfo[y + 1].y, s0 + cbn);
                reinterpret_cast<uint4*>(desc_w)[2 * (size_t)cc] = make_uint4(y, kk, ri.w, ri.z);
                desc_w[8 * (size_t)cc + 4] = s0;
                desc_w[8 * (size_t)cc + 5] = s1;
                desc_w[8 * (size_t)cc + 6] = dst;  // first owner
                if (kk > 0) desc_w[8 * (size_t)(cc - 1) + 7] = ex < s0 ? dst + 1 : dst;  // owner end of the chunk before
            }
        }
        k = kn;
        __syncthreads();  // the next chunk rewrites the staging arrays
    }
}

// ---- columns pass ------------------------------------------------------------------------------------------------
// chunk c of the columns pass: row y, its chunk kk, instance slots [s0, s1), owners (row entries) e_lo .. e_lo + nr - 1
struct ColChunk {
    uint32_t y, kk, nch, cb, s0, s1, e_lo, nr;
};
// desc_b[c] = {y, kk, chunks of the row, row's first chunk}, {s0, s1, first owner, owner end} (rows_scatter_kernel,
// rows_info)
__device__ __forceinline__ ColChunk col_chunk(const BinArgs& a, uint32_t c)
{
    const uint4 d0 = a.desc_b[2 * (size_t)c], d1 = a.desc_b[2 * (size_t)c + 1];
    return ColChunk{d0.x, d0.y, d0.z, d0.w, d1.x, d1.y, d1.z, d1.w - d1.z};
}
// index of (row y, column x, chunk kk) in the tile-major [tile][chunk] counts
__device__ __forceinline__ size_t col_index(const ColChunk& k, uint32_t gx, uint32_t x)
{
    return (size_t)k.cb * gx + (size_t)x * k.nch + k.kk;
}

// Per column chunk (grid-stride): the instance counts per tile column from a difference array. Latency-bound, so
// every load of a chunk is issued before any is used: the owners' words for the first HP x 256 owners at once, and
// the next chunk's descriptor while this one is counted.
__global__ __launch_bounds__(RB_THREADS) void cols_hist_kernel(BinArgs a)
{
    constexpr int HP = 4;
    __shared__ int s_diff[BIN_MAX_GRID + 1];
    __shared__ uint32_t s_wave[RB_WAVES];
    const uint32_t tid = threadIdx.x, gx = a.gx, C = a.words[1];
    const ChunkRange cr = xcd_chunks(C);
    if (C == 0) return;  // no live chunk: desc_b has no entry to prefetch
    ColChunk k = col_chunk(a, min(cr.first, C - 1u));
    for (uint32_t c = cr.first; c < cr.end; c += cr.step) {
        const ColChunk kn = col_chunk(a, min(c + cr.step, C - 1u));
        uint32_t ex[HP], ew[HP];
#pragma unroll
        for (int j = 0; j < HP; ++j) {
            const uint32_t i = tid + j * RB_THREADS;
            if (i < k.nr) {
                ex[j] = a.ent_ex[k.e_lo + i];
                ew[j] = a.ent_w[k.e_lo + i];
            }
        }
        for (uint32_t x = tid; x <= gx; x += RB_THREADS) s_diff[x] = 0;
        __syncthreads();
        auto add = [&](uint32_t e_x, uint32_t e_w) {
            const uint32_t wd = e_w & 0xFFFFu, x0 = e_w >> 16;
            const uint32_t ja = max(k.s0, e_x) - e_x, jb = min(k.s1, e_x + wd) - e_x;
            atomicAdd(&s_diff[x0 + ja], 1);
            atomicAdd(&s_diff[x0 + jb], -1);
        };
#pragma unroll
        for (int j = 0; j < HP; ++j)
            if (tid + j * RB_THREADS < k.nr) add(ex[j], ew[j]);
        for (uint32_t i = tid + HP * RB_THREADS; i < k.nr; i += RB_THREADS) add(a.ent_ex[k.e_lo + i], a.ent_w[k.e_lo + i]);
        __syncthreads();
        diff_to_counts<RB_THREADS>(s_diff, gx, s_wave);
        for (uint32_t x = tid; x < gx; x += RB_THREADS) a.hist_b[col_index(k, gx, x)] = (uint32_t)s_diff[x];
        k = kn;
        __syncthreads();
    }
}

// the slots of one round: column, point-list word (Gaussian | band mask << PL_GID_BITS); STAGED: every owner's band
// intervals and Gaussian are in LDS (a chunk-uniform choice, so the loads stay plain LDS reads), else each slot derives
// its owner's intervals from bin_rec itself
template <bool STAGED, class G>
__device__ __forceinline__ void col_expand(const BinArgs& a, const ColChunk& k, const uint16_t* s_own,
                                           const uint32_t* s_xoff, const uint4* s_iv, const uint32_t* s_gid,
                                           uint32_t (&d)[G::ROUNDS],
                                           uint32_t (&val)[G::ROUNDS], bool (&valid)[G::ROUNDS])
{
    const uint32_t lane = threadIdx.x & 63u, w = threadIdx.x >> 6;
#pragma unroll
    for (int r = 0; r < G::ROUNDS; ++r) {
        const uint32_t j = w * G::PER_WAVE + 64u * r + lane, s = k.s0 + j;
        valid[r] = s < k.s1;
        d[r] = 0;
        val[r] = 0;
        if (valid[r]) {
            const uint32_t o = s_own[j];
            const uint32_t x = s + s_xoff[o];
            uint4 iv;
            uint32_t gid;
            if (STAGED) {
                iv = s_iv[o];
                gid = s_gid[o];
            } else {
                gid = a.ent_gid[k.e_lo + o];
                iv = band_row_intervals(a.bin_rec[2 * (size_t)gid], a.bin_rec[2 * (size_t)gid + 1], k.y, 0u, a.gx);
            }
            d[r] = x;
            val[r] = gid | (band_mask_of_intervals(iv, x) << PL_GID_BITS);
        }
    }
}

template <int BITS, class G>
__global__ __launch_bounds__(G::THREADS) void cols_scatter_kernel(BinArgs a)
{
    // phase 1 (expansion): per owner, x0 minus its first instance slot (slot s is column s + s_xoff), and, when the
    // owners fit, each one's reachable columns per band of this row (band_row_intervals: computed once per row entry,
    // not once per instance) and its Gaussian; phase 2 (write-out): the slots' point-list words and columns in column
    // order, in the same storage
    constexpr uint32_t CB_OWN = G::N / 2;  // owners staged in LDS (C's 2048-slot chunks have ~600, E's 4096 ~650)
    constexpr size_t PH1 = G::N * sizeof(uint32_t) + CB_OWN * (sizeof(uint4) + sizeof(uint32_t));
    constexpr size_t PH2 = G::N * (sizeof(uint32_t) + sizeof(uint16_t));
    __shared__ uint4 s_raw[(PH1 > PH2 ? PH1 : PH2) / sizeof(uint4)];
    uint4* s_iv = s_raw;
    uint32_t* s_gid = reinterpret_cast<uint32_t*>(s_raw + CB_OWN);
    uint32_t* s_xoff = s_gid + CB_OWN;
    __shared__ __attribute__((aligned(16))) uint16_t s_own[G::N];
    __shared__ uint32_t s_whist[G::WAVES][1 << BITS];
    __shared__ uint32_t s_dstart[1 << BITS];
    __shared__ uint32_t s_gbase[1 << BITS];
    __shared__ uint32_t s_wave[G::WAVES];
    static_assert(BITS != 8 || sizeof(s_raw) >= G::WAVES * 256 * sizeof(uint64_t), "peer tables fit s_raw");
    const uint32_t tid = threadIdx.x, gx = a.gx, C = a.words[1];
    const uint32_t L = live_L(a.counters, a.cap);
    uint32_t* point_list = reinterpret_cast<uint32_t*>(a.binning + canonical_list_offset(L));
    // software pipeline: the next chunk's descriptor, count bases and its first PF x 256 owners' entries and band
    // constants are loaded into registers while the current chunk is expanded and ranked (more would cost the VGPRs
    // of a fourth block per CU); staged owners past those are loaded when staged
    constexpr int PF = 2;
    static_assert(PF * G::THREADS <= CB_OWN, "prefetched owners are staged owners");
    typedef float f4v __attribute__((ext_vector_type(4)));  // native vectors: the prefetch stays in registers
    constexpr int GBP = ((1 << BITS) + G::THREADS - 1) / G::THREADS;  // per-column count bases per thread
    uint32_t p_ex[PF], p_ew[PF], p_gid[PF], p_gb[GBP];
    f4v p_ba[PF], p_bb[PF];
    const f4v* bin_rec_v = reinterpret_cast<const f4v*>(a.bin_rec);
#define OMR_CS_LOAD_ENTRIES(q)                                                 \
    _Pragma("unroll") for (int j = 0; j < PF; ++j)                             \
    {                                                                          \
        const uint32_t i_ = tid + j * G::THREADS;                              \
        if ((q).nr <= CB_OWN && i_ < (q).nr) {                           \
            p_ex[j] = a.ent_ex[(q).e_lo + i_];                                 \
            p_ew[j] = a.ent_w[(q).e_lo + i_];                                  \
            p_gid[j] = a.ent_gid[(q).e_lo + i_];                               \
        }                                                                      \
    }                                                                          \
    _Pragma("unroll") for (int j = 0; j < GBP; ++j)                            \
    {                                                                          \
        const uint32_t x_ = tid + j * G::THREADS;                              \
        if (x_ < gx) p_gb[j] = a.hist_b[col_index((q), gx, x_)];               \
    }
#define OMR_CS_LOAD_CONSTS(q)                                                  \
    _Pragma("unroll") for (int j = 0; j < PF; ++j)                             \
    {                                                                          \
        const uint32_t i_ = tid + j * G::THREADS;                              \
        if ((q).nr <= CB_OWN && i_ < (q).nr) {                           \
            p_ba[j] = bin_rec_v[2 * (size_t)p_gid[j]];                         \
            p_bb[j] = bin_rec_v[2 * (size_t)p_gid[j] + 1];                     \
        }                                                                      \
    }
    const ChunkRange cr = xcd_chunks(C);
    uint32_t c = cr.first, it = 0;
    if (C == 0) return;  // no live chunk: desc_b has no entry to prefetch
    ColChunk k = col_chunk(a, min(c, C - 1u));
    if (c < cr.end) {
        OMR_CS_LOAD_ENTRIES(k)
        OMR_CS_LOAD_CONSTS(k)
    }
    for (; c < cr.end; c += cr.step, ++it) {
        BSTAMP(it, 0);
        const uint32_t cn = c + cr.step;
        const ColChunk kn = col_chunk(a, min(cn, C - 1u));  // the next chunk's descriptor, in flight meanwhile
        const bool staged = k.nr <= CB_OWN;  // chunk-uniform
        reinterpret_cast<uint4*>(s_own)[tid] = make_uint4(0u, 0u, 0u, 0u);
        __syncthreads();
        if (staged) {
#pragma unroll
            for (int j = 0; j < PF; ++j) {
                const uint32_t i = tid + j * G::THREADS;
                if (i < k.nr) {
                    s_xoff[i] = (p_ew[j] >> 16) - p_ex[j];  // modular
                    if (p_ex[j] >= k.s0) s_own[p_ex[j] - k.s0] = (uint16_t)i;  // distinct first slots (width >= 1)
                    const f4v ba = p_ba[j], bb = p_bb[j];
                    s_iv[i] = band_row_intervals(make_float4(ba.x, ba.y, ba.z, ba.w), make_float4(bb.x, bb.y, bb.z, bb.w),
                                                 k.y, 0u, gx);
                    s_gid[i] = p_gid[j];
                }
            }
            for (uint32_t i = tid + PF * G::THREADS; i < k.nr; i += G::THREADS) {
                const uint32_t e = k.e_lo + i, ex = a.ent_ex[e], gid = a.ent_gid[e];
                s_xoff[i] = (a.ent_w[e] >> 16) - ex;
                if (ex >= k.s0) s_own[ex - k.s0] = (uint16_t)i;
                s_iv[i] = band_row_intervals(a.bin_rec[2 * (size_t)gid], a.bin_rec[2 * (size_t)gid + 1], k.y, 0u, gx);
                s_gid[i] = gid;
            }
        } else {
            for (uint32_t i = tid; i < k.nr; i += G::THREADS) {
                const uint32_t e = k.e_lo + i;
                const uint32_t ex = a.ent_ex[e];
                s_xoff[i] = (a.ent_w[e] >> 16) - ex;
                if (ex >= k.s0) s_own[ex - k.s0] = (uint16_t)i;
            }
        }
#pragma unroll
        for (int j = 0; j < GBP; ++j)
            if (tid + j * G::THREADS < gx) s_gbase[tid + j * G::THREADS] = p_gb[j];
        __syncthreads();
        if (cn < cr.end) {
            OMR_CS_LOAD_ENTRIES(kn)
        }
        BSTAMP(it, 1);
        owner_fill<G>(s_own, s_wave);
        BSTAMP(it, 2);
        uint32_t d[G::ROUNDS], val[G::ROUNDS], lp[G::ROUNDS];
        bool valid[G::ROUNDS];
        if (staged) col_expand<true, G>(a, k, s_own, s_xoff, s_iv, s_gid, d, val, valid);
        else col_expand<false, G>(a, k, s_own, s_xoff, s_iv, s_gid, d, val, valid);
        if (cn < cr.end) {
            OMR_CS_LOAD_CONSTS(kn)
        }
        BSTAMP(it, 3);
        // its barriers end the expansion's reads of s_raw, which then holds the peer tables
        rank_items<BITS, G>(d, valid, lp, s_whist, s_dstart, s_wave,
                            BITS == 8 ? reinterpret_cast<uint64_t*>(s_raw) : nullptr);
        BSTAMP(it, 4);
        uint32_t* s_v = reinterpret_cast<uint32_t*>(s_raw);
        uint16_t* s_x = reinterpret_cast<uint16_t*>(s_v + G::N);
#pragma unroll
        for (int r = 0; r < G::ROUNDS; ++r)
            if (valid[r]) {
                s_v[lp[r]] = val[r];
                s_x[lp[r]] = (uint16_t)d[r];
            }
        __syncthreads();
        BSTAMP(it, 5);
        const uint32_t nvalid = k.s1 - k.s0;
        for (uint32_t j = tid; j < nvalid; j += G::THREADS) {
            const uint32_t x = s_x[j];
            point_list[s_gbase[x] + (j - s_dstart[x])] = s_v[j];
        }
        // identifyTileRanges from the counts: the row's first chunk writes its tiles' ranges; empty tiles keep the
        // {0, 0} preprocess wrote, as the reference leaves them (rasterizer_impl.cu:145-167 writes boundaries only)
        if (k.kk == 0)
            for (uint32_t x = tid; x < gx; x += G::THREADS) {
                const size_t i = col_index(k, gx, x);
                const uint32_t b0 = a.hist_b[i], b1 = a.hist_b[i + k.nch];
                if (b1 != b0) a.ranges[(size_t)k.y * gx + x] = make_uint2(b0, b1);
            }
        BSTAMP(it, 6);
        k = kn;
        __syncthreads();  // the next chunk rewrites the staging arrays
        BSTAMP(it, 7);
    }
#undef OMR_CS_LOAD_ENTRIES
#undef OMR_CS_LOAD_CONSTS
}

}  // namespace

#ifdef OMR_BIN_STAMPS
extern "C" int omr_debug_bin_stamps(uint64_t* dst, size_t bytes)
{
    return (int)hipMemcpyFromSymbol(dst, HIP_SYMBOL(g_bin_stamps), std::min(bytes, sizeof(g_bin_stamps)));
}
#endif

// scratch of the row binning for a binning capacity of `cap` instances (BinningState::carve)
size_t bin_chunks_r(size_t cap) { return div_up(cap, RB_N) + 1; }
uint32_t bin_cols_shift(size_t cap)
{
    static const uint32_t forced = [] {  // OMR_BIN_COLS_SHIFT=9..12 (A/B runs): the columns-pass chunk for every view
        const char* v = std::getenv("OMR_BIN_COLS_SHIFT");
        const int k = v ? std::atoi(v) : 0;
        return (k >= 9 && k <= 12) ? (uint32_t)k : 0u;
    }();
    if (forced) return forced;
    // 1024-slot chunks below 2 M instances (configs A, B: +0.5-0.8 %, profiles/r06k_ab_{A,B}.txt); C's 2048 (1024:
    // -1 %, 512: -2.6 %, r06k_ab_C.txt), E's 4096
    return cap >= ((size_t)1 << 25) ? 12u : cap >= ((size_t)1 << 21) ? 11u : 10u;
}
size_t bin_chunks_b(size_t cap, uint32_t gy) { return (div_up(cap, (size_t)1 << bin_cols_shift(cap))) + gy + 1; }

void launch_row_binning(const BinArgs& a_in, hipStream_t s)
{
    BinArgs a = a_in;
    a.cb_shift = bin_cols_shift(a.cap);
    const uint32_t cr = (uint32_t)a.chunks_r, cbk = (uint32_t)a.chunks_b;
    // look-back words of the two scans, zeroed by rows_hist_kernel; grids and scans are sized for the capacity (capped
    // grid-stride kernels and persistent scans), the kernels stop at the live lengths (words[])
    const size_t nr_hist = 2 * (size_t)a.gy * cr, nb_hist = (size_t)cbk * a.gx;
    const size_t zr = scan_status_words(nr_hist), zb = scan_status_words(nb_hist);
    uint32_t* st_r = a.zero;
    uint32_t* st_b = st_r + zr;
    a.nzero = zr + zb;
    const uint32_t gh_r = std::min(cr, BIN_GRID_HIST), gs_r = std::min(cr, BIN_GRID_SCATTER);
    const uint32_t gh_b = std::min(cbk, BIN_GRID_HIST);
    rows_hist_kernel<<<gh_r, RB_THREADS, 0, s>>>(a);
    launch_exclusive_scan(a.hist_r, a.hist_r, nr_hist, a.words + 2, st_r, a.err, s);
    if (a.gy <= 256) rows_scatter_kernel<8><<<gs_r, RB_THREADS, 0, s>>>(a);
    else rows_scatter_kernel<10><<<gs_r, RB_THREADS, 0, s>>>(a);
    cols_hist_kernel<<<gh_b, RB_THREADS, 0, s>>>(a);
    launch_exclusive_scan(a.hist_b, a.hist_b, nb_hist, a.words + 3, st_b, a.err, s);
    auto scatter = [&](auto geo) {
        using G = decltype(geo);
        const uint32_t g = std::min(cbk, BIN_GRID_SCATTER * (uint32_t)ColGeoS::THREADS / (uint32_t)G::THREADS);
        if (a.gx <= 256) cols_scatter_kernel<8, G><<<g, G::THREADS, 0, s>>>(a);
        else cols_scatter_kernel<10, G><<<g, G::THREADS, 0, s>>>(a);
    };
    if (a.cb_shift == 12) scatter(ColGeoL{});
    else if (a.cb_shift == 11) scatter(ColGeoS{});
    else if (a.cb_shift == 10) scatter(ColGeoM{});
    else scatter(ColGeoT{});
}

}  // namespace omr
