// lane_study.cpp — CPU study of render-kernel lane mappings (profiles/lane_study.py dumps the oracle's forward state).
//
// Counts, per lane mapping, the wave steps the render kernels would issue and how many lanes of each step hold a
// contributing (pixel, instance) pair:
//   band16x4  the current mapping (tile_wave.h): per 16x4 band, every instance whose ellipse reaches the band is
//             evaluated by all 64 lanes (one pixel each), until the band's pixels are all done (forward) / up to the
//             band's last contributor (backward);
//   blk4x4    16-lane groups, each owning one 4x4 block of a 16x4 band and walking its own list: a step advances all
//             four groups by one instance of their own list, so a band costs max over its 4 blocks of the list length;
//   q8x8      the same with the four 4x4 blocks of an 8x8 quadrant as the groups (a round = one quadrant);
//   blk4x4_bbox  blk4x4 with the block lists the render kernel can form cheaply: the binning's exact 16x4 band mask
//             times the columns the ellipse's x-extent meets;
//   quad8x8   the current algorithm with 8x8 quadrants in place of 16x4 bands: per quadrant, every instance whose
//             ellipse reaches it is evaluated by all 64 lanes (one pixel each; one instance per step, as today).
// Input: raw little-endian arrays written by lane_study.py into a directory.
#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <string>
#include <vector>

template <typename T> static std::vector<T> load(const std::string& path)
{
    FILE* f = std::fopen(path.c_str(), "rb");
    if (!f) { std::perror(path.c_str()); std::exit(1); }
    std::fseek(f, 0, SEEK_END);
    const long n = std::ftell(f);
    std::fseek(f, 0, SEEK_SET);
    std::vector<T> v(n / sizeof(T));
    if (std::fread(v.data(), 1, n, f) != (size_t)n) { std::perror("read"); std::exit(1); }
    std::fclose(f);
    return v;
}

int main(int argc, char** argv)
{
    if (argc < 2) { std::fprintf(stderr, "usage: lane_study DIR\n"); return 1; }
    const std::string d = argv[1];
    const auto dims = load<int32_t>(d + "/dims.bin");  // W, H
    const int W = dims[0], H = dims[1];
    const auto m2 = load<float>(d + "/means2D.bin");
    const auto co = load<float>(d + "/conic_opacity.bin");
    const auto pl = load<uint32_t>(d + "/point_list.bin");
    const auto rg = load<uint32_t>(d + "/ranges.bin");
    const int gx = (W + 15) / 16, gy = (H + 15) / 16;
    // totals: [mapping][fwd/bwd] steps, contributing pairs
    double steps[5][2] = {}, evalpairs[5][2] = {}, contrib = 0, fwd_live = 0;
    // band pairs (0, 1) and (2, 3) of a tile (one lane's two pixels of a pair share a column): per direction, the
    // (instance, pair) evaluations that need both bands and those that need one (packed-math study)
    double pair_both[2] = {0, 0}, pair_one[2] = {0, 0};
#pragma omp parallel for schedule(dynamic, 16) reduction(+ : contrib, fwd_live)
    for (int t = 0; t < gx * gy; ++t) {
        const int tx = t % gx, ty = t / gx;
        const uint32_t r0 = rg[2 * t], r1 = rg[2 * t + 1], n = r1 - r0;
        if (!n) continue;
        // per pixel (16x16, row-major): reach bits per instance, done position (forward) and last contributor
        std::vector<uint8_t> reach((size_t)n * 256, 0);
        int done[256], last[256];
        for (int p = 0; p < 256; ++p) {
            const int px = tx * 16 + p % 16, py = ty * 16 + p / 16;
            done[p] = -1;
            last[p] = 0;
            if (px >= W || py >= H) continue;
            double T = 1.0;
            done[p] = (int)n - 1;
            for (uint32_t k = 0; k < n; ++k) {
                const uint32_t g = pl[r0 + k];
                const double dx = m2[2 * g] - px, dy = m2[2 * g + 1] - py;
                const double* c = nullptr;
                (void)c;
                const double a = co[4 * g], b = co[4 * g + 1], cc = co[4 * g + 2], o = co[4 * g + 3];
                const double power = -0.5 * (a * dx * dx + cc * dy * dy) - b * dx * dy;
                if (power > 0) continue;
                const double alpha = std::min(0.99, o * std::exp(power));
                if (alpha < 1.0 / 255.0) continue;
                const double tt = T * (1 - alpha);
                reach[(size_t)k * 256 + p] = 1;
                if (tt < 1e-4) { done[p] = (int)k; break; }
                T = tt;
                last[p] = (int)k + 1;
            }
        }
        for (int p = 0; p < 256; ++p)
            for (uint32_t k = 0; k < n && (int)k < last[p]; ++k) contrib += reach[(size_t)k * 256 + p];
        // groups of 16 pixels: band b (rows 4b..4b+3, all 16 columns) = 4 blocks; block (bx, by) of 4x4
        // per instance: the x-extent of its alpha >= 1/255 ellipse (a bound the render kernel can form from the record:
        // a dx^2 + 2 b dx dy + c dy^2 <= 2 ln(255 o) reaches |dx| <= sqrt(2 ln(255 o) c / (ac - b^2)))
        std::vector<double> xlo(n), xhi(n);
        for (uint32_t k = 0; k < n; ++k) {
            const uint32_t g = pl[r0 + k];
            const double a = co[4 * g], b = co[4 * g + 1], cc = co[4 * g + 2], o = co[4 * g + 3];
            const double R = 2.0 * std::log(255.0 * o);
            const double ex = R > 0 ? std::sqrt(R * cc / (a * cc - b * b)) : -1.0;
            xlo[k] = m2[2 * g] - ex;
            xhi[k] = m2[2 * g] + ex;
        }
        // bbox mode: an instance counts for a 4x4 block when it reaches the block's 16x4 band (the binning's exact band
        // mask) and its x-extent meets the block's four columns
        int bbox_band = -1, bbox_x0 = 0;
        auto count = [&](const std::vector<int>& pix, int& fsteps, int& bsteps, int& fpairs, int& bpairs) {
            int fend = -1, bend = 0;  // forward: while any pixel is live; backward: up to the last contributor
            for (int p : pix) { fend = std::max(fend, done[p]); bend = std::max(bend, last[p]); }
            fsteps = bsteps = fpairs = bpairs = 0;
            for (int k = 0; k <= fend || k < bend; ++k) {
                bool any = false;
                if (bbox_band >= 0) {
                    bool band = false;
                    for (int r = 0; r < 4 && !band; ++r)
                        for (int c = 0; c < 16 && !band; ++c) band = reach[(size_t)k * 256 + (4 * bbox_band + r) * 16 + c];
                    any = band && xhi[k] >= tx * 16 + bbox_x0 && xlo[k] <= tx * 16 + bbox_x0 + 3;
                }
                int live_f = 0, live_b = 0;
                for (int p : pix) {
                    if (!reach[(size_t)k * 256 + p]) continue;
                    if (bbox_band < 0) any = true;
                    if (k <= done[p] && k < (int)n) live_f += (k < last[p] || k == done[p]);
                    live_b += k < last[p];
                }
                if (!any) continue;
                if (k <= fend) { ++fsteps; fpairs += live_f; }
                if (k < bend) { ++bsteps; bpairs += live_b; }
            }
        };
        double ls[5][2] = {}, lp[5][2] = {};
        {
            // per band: window ends and reach of each instance
            int fe[4], be[4];
            for (int b = 0; b < 4; ++b) {
                fe[b] = -1, be[b] = 0;
                for (int r = 0; r < 4; ++r)
                    for (int c = 0; c < 16; ++c) {
                        const int p = (4 * b + r) * 16 + c;
                        fe[b] = std::max(fe[b], done[p]);
                        be[b] = std::max(be[b], last[p]);
                    }
            }
            double both[2] = {0, 0}, one[2] = {0, 0};
            for (uint32_t k = 0; k < n; ++k) {
                bool rb[4];
                for (int b = 0; b < 4; ++b) {
                    rb[b] = false;
                    for (int q = 0; q < 64 && !rb[b]; ++q) rb[b] = reach[(size_t)k * 256 + 64 * b + q];
                }
                for (int pr = 0; pr < 2; ++pr) {
                    const int b0 = 2 * pr, b1 = b0 + 1;
                    for (int dir = 0; dir < 2; ++dir) {
                        const bool n0 = rb[b0] && (dir == 0 ? (int)k <= fe[b0] : (int)k < be[b0]);
                        const bool n1 = rb[b1] && (dir == 0 ? (int)k <= fe[b1] : (int)k < be[b1]);
                        if (n0 && n1) both[dir] += 1;
                        else if (n0 || n1) one[dir] += 1;
                    }
                }
            }
#pragma omp critical
            for (int dir = 0; dir < 2; ++dir) { pair_both[dir] += both[dir]; pair_one[dir] += one[dir]; }
        }
        // band16x4
        for (int b = 0; b < 4; ++b) {
            std::vector<int> pix;
            for (int r = 0; r < 4; ++r)
                for (int c = 0; c < 16; ++c) pix.push_back((4 * b + r) * 16 + c);
            int fs, bs, fp, bp;
            count(pix, fs, bs, fp, bp);
            ls[0][0] += fs; ls[0][1] += bs; lp[0][0] += fp; lp[0][1] += bp;
        }
        // quad8x8: the band algorithm on 8x8 quadrants
        for (int q = 0; q < 4; ++q) {
            std::vector<int> pix;
            for (int y = 0; y < 8; ++y)
                for (int x = 0; x < 8; ++x) pix.push_back((8 * (q / 2) + y) * 16 + 8 * (q % 2) + x);
            int fs, bs, fp, bp;
            count(pix, fs, bs, fp, bp);
            ls[4][0] += fs; ls[4][1] += bs; lp[4][0] += fp; lp[4][1] += bp;
        }
        // blk4x4 rounds = bands; q8x8 rounds = quadrants
        for (int mode = 1; mode < 4; ++mode)
            for (int r = 0; r < 4; ++r) {
                int mf = 0, mb = 0;
                for (int gidx = 0; gidx < 4; ++gidx) {
                    int bx, by;
                    bbox_band = mode == 3 ? r : -1;
                    bbox_x0 = 4 * gidx;
                    if (mode != 2) { bx = gidx; by = r; }
                    else { bx = (r % 2) * 2 + gidx % 2; by = (r / 2) * 2 + gidx / 2; }
                    std::vector<int> pix;
                    for (int y = 0; y < 4; ++y)
                        for (int x = 0; x < 4; ++x) pix.push_back((4 * by + y) * 16 + 4 * bx + x);
                    int fs, bs, fp, bp;
                    count(pix, fs, bs, fp, bp);
                    mf = std::max(mf, fs);
                    mb = std::max(mb, bs);
                    lp[mode][0] += fp; lp[mode][1] += bp;
                }
                ls[mode][0] += mf; ls[mode][1] += mb;
            }
        bbox_band = -1;
#pragma omp critical
        for (int m = 0; m < 5; ++m)
            for (int k = 0; k < 2; ++k) { steps[m][k] += ls[m][k]; evalpairs[m][k] += lp[m][k]; }
    }
    const char* names[5] = {"band16x4", "blk4x4", "q8x8", "blk4x4_bbox", "quad8x8"};
    std::printf("{\"W\": %d, \"H\": %d, \"contributing_pairs\": %.0f", W, H, contrib);
    for (int m = 0; m < 5; ++m)
        std::printf(", \"%s\": {\"fwd_steps\": %.0f, \"bwd_steps\": %.0f, \"fwd_lane_use\": %.4f, \"bwd_lane_use\": %.4f}",
                    names[m], steps[m][0], steps[m][1], evalpairs[m][0] / (64.0 * steps[m][0]),
                    evalpairs[m][1] / (64.0 * steps[m][1]));
    std::printf(", \"band_pairs\": {\"fwd_both\": %.0f, \"fwd_one\": %.0f, \"bwd_both\": %.0f, \"bwd_one\": %.0f}",
                pair_both[0], pair_one[0], pair_both[1], pair_one[1]);
    std::printf("}\n");
    (void)fwd_live;
    return 0;
}
