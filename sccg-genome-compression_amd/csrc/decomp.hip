// decomp.hip -- reconstruction of the target FASTA from the record text (decompression.cpp).
//
//   line split                  decompression.cpp:66-101
//   run-line parse              decompression.cpp:126-207 ("(d,len)" / "d," items, running start)
//   token decode                decompression.cpp:210-236 ("(dp,l)" -> ref[p, p+l), literals)
//   N insertion, lowercase      decompression.cpp:241-262
//   50-column output            decompression.cpp:266-274, :322
//
// All of it is data-parallel: item starts are found with a scan of "last parenthesis" positions,
// numbers are parsed one item per thread, running starts / absolute p are prefix sums, output
// offsets are prefix sums, and the final FASTA is written position-by-position with N and
// lowercase membership found by binary search over the (sorted, disjoint) run lists.
// Inputs the reference's own compressor can produce are handled exactly; text outside that
// grammar is reported as SCCG_E_PARSE instead of reproducing the reference's undefined paths.
#include <cstdlib>

#include "internal.h"
#include "decomp.h"

namespace {

__device__ __forceinline__ bool is_num(uint8_t c) { return (c >= '0' && c <= '9') || c == '-' || c == '+'; }

// stoi on [s, e): optional sign then digits, all of [s,e) consumed; returns false otherwise
__device__ __forceinline__ bool parse_int(const uint8_t* s, int64_t n, int64_t a, int64_t e, int64_t* v) {
    if (a >= e) return false;
    bool neg = false;
    if (s[a] == '-' || s[a] == '+') { neg = s[a] == '-'; a++; }
    if (a >= e || e - a > 10) return false;
    int64_t x = 0;
    for (int64_t i = a; i < e; i++) {
        const uint8_t c = s[i];
        if (c < '0' || c > '9') return false;
        x = x * 10 + (c - '0');
    }
    x = neg ? -x : x;
    if (x > INT32_MAX || x < INT32_MIN) return false;
    *v = x;
    (void)n;
    return true;
}

// every '\n' of the record text into nl[0, NL_CAP) in any order, their count in *cnt (a record
// file holds 2-3 of them; the caller falls back to ordered searches when there are more)
__global__ void k_newlines(const uint8_t* __restrict__ s, int64_t n, unsigned long long* __restrict__ cnt,
                           int64_t* __restrict__ nl) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
        if (s[i] == '\n') {
            const unsigned long long k = atomicAdd(cnt, 1ull);
            if (k < (unsigned long long)DC_NL_CAP) nl[k] = i;
        }
}

// positions of '(' / ')' -> value i, else -1 (for a max-scan: last parenthesis at or before i)
__global__ void k_paren_pos(const uint8_t* __restrict__ s, int64_t n, int64_t* __restrict__ v) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
        v[i] = (s[i] == '(' || s[i] == ')') ? i : -1;
}

// ---------------------------------------------------------------------------------------------
// run lines: item start flags (exclusive max-scan `lp` = last paren strictly before i)
// ---------------------------------------------------------------------------------------------
__device__ __forceinline__ bool run_item_start(const uint8_t* s, int64_t i, int64_t lp_excl) {
    const uint8_t c = s[i];
    if (c == '(') return true;
    if (!is_num(c)) return false;
    const bool inside = lp_excl >= 0 && s[lp_excl] == '(';
    return !inside && (i == 0 || !is_num(s[i - 1]));
}

__global__ void k_run_items_flag(const uint8_t* __restrict__ s, int64_t n, const int64_t* __restrict__ lp,
                                 int64_t* __restrict__ flag, int32_t* __restrict__ err) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        const bool st = run_item_start(s, i, lp[i]);
        flag[i] = st;
        // bytes outside any item must be ',' (a ')' closes a tuple)
        const uint8_t c = s[i];
        const bool inside = (lp[i] >= 0 && s[lp[i]] == '(') || c == '(' || c == ')';
        if (!inside && !is_num(c) && c != ',') atomicOr(err, 1);
    }
}

__global__ void k_run_items_parse(const uint8_t* __restrict__ s, int64_t n, const int64_t* __restrict__ lp,
                                  const int64_t* __restrict__ rank, int64_t* __restrict__ dlt,
                                  int32_t* __restrict__ len, int32_t* __restrict__ err) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        if (!run_item_start(s, i, lp[i])) continue;
        const int64_t r = rank[i];
        int64_t d = 0, l = 1;
        bool ok;
        if (s[i] == '(') {
            int64_t comma = -1, close = -1;
            for (int64_t q = i + 1; q < n && q < i + 32; q++) {
                if (s[q] == ',' && comma < 0) comma = q;
                if (s[q] == ')') { close = q; break; }
                if (s[q] == '(') break;
            }
            ok = comma > 0 && close > comma && parse_int(s, n, i + 1, comma, &d) && parse_int(s, n, comma + 1, close, &l);
            // a ',' right after ')' is consumed by the reference parser (decompression.cpp:143-144)
        } else {
            int64_t e = i;
            while (e < n && is_num(s[e])) e++;
            ok = (e == n || s[e] == ',') && parse_int(s, n, i, e, &d);
        }
        if (!ok || l < 0) { atomicOr(err, 1); continue; }
        dlt[r] = d;
        len[r] = (int32_t)l;
    }
}

// ---------------------------------------------------------------------------------------------
// run lines, tiled: one wave per 1 KiB tile, 16 bytes per lane, the tile staged in LDS with the 32
// bytes before it and the 64 after it (every byte read of the parse is an LDS read; coalesced HBM
// loads once per pass).  A run line's parentheses only open "(d,len)" items of at most 25 bytes, so
// the "inside an item" state at a lane's first byte follows from the last parenthesis before it:
// in the lanes before it (a wave max-scan), else in the 32 bytes before the tile (text outside the
// compressor's grammar is flagged by the item parses either way).  Three launches per line instead
// of a parenthesis max-scan, an item-rank scan and three prefix sums (decompression.cpp:126-207 per
// item, running start, sorted).
// ---------------------------------------------------------------------------------------------
#ifndef SCCG_RL_LANE
#define SCCG_RL_LANE 8   // (16: ~5 us slower on the chr1 reconstruction, more serial bytes per lane)
#endif
constexpr int RL_LANE = SCCG_RL_LANE, RL_TILE = 64 * RL_LANE, RL_BEHIND = 32, RL_AHEAD = 64;
constexpr int RL_STAGE = RL_BEHIND + RL_TILE + RL_AHEAD;

// the wave's staged bytes: global positions [t0 - RL_BEHIND, t0 + tile + RL_AHEAD), 0 outside [0, n)
struct RlView {
    const uint8_t* b;
    int64_t t0, n, tile;
    __device__ __forceinline__ uint8_t at(int64_t i) const { return b[i - t0 + RL_BEHIND]; }
    __device__ __forceinline__ int64_t lim() const { return t0 + tile + RL_AHEAD; }
};

template <int TILE>
__device__ __forceinline__ RlView rl_stage(const uint8_t* __restrict__ s, int64_t n, int64_t t0, uint8_t* st) {
    for (int k = lane_id(); k < RL_BEHIND + TILE + RL_AHEAD; k += 64) {
        const int64_t g = t0 - RL_BEHIND + k;
        st[k] = (g >= 0 && g < n) ? s[g] : (uint8_t)0;
    }
    wave_sync();
    return RlView{st, t0, n, TILE};
}

__device__ __forceinline__ bool parse_int_v(const RlView& v, int64_t a, int64_t e, int64_t* out) {
    if (a >= e) return false;
    bool neg = false;
    if (v.at(a) == '-' || v.at(a) == '+') { neg = v.at(a) == '-'; a++; }
    if (a >= e || e - a > 10) return false;
    int64_t x = 0;
    for (int64_t i = a; i < e; i++) {
        const uint8_t c = v.at(i);
        if (c < '0' || c > '9') return false;
        x = x * 10 + (c - '0');
    }
    x = neg ? -x : x;
    if (x > INT32_MAX || x < INT32_MIN) return false;
    *out = x;
    return true;
}

// one item at i (inside the tile): "(d,l)" or a bare "d" followed by ',' or the end
// (decompression.cpp:126-164); a bare number running past the staged bytes is not the compressor's
__device__ __forceinline__ bool rl_item(const RlView& v, int64_t i, int64_t* d, int64_t* l) {
    const int64_t n = v.n, lim = v.lim();
    *l = 1;
    if (v.at(i) == '(') {
        int64_t comma = -1, close = -1;
        for (int64_t q = i + 1; q < n && q < i + 32; q++) {
            const uint8_t c = v.at(q);
            if (c == ',' && comma < 0) comma = q;
            if (c == ')') { close = q; break; }
            if (c == '(') break;
        }
        return comma > 0 && close > comma && parse_int_v(v, i + 1, comma, d) && parse_int_v(v, comma + 1, close, l) &&
               *l >= 0;
    }
    int64_t e = i;
    while (e < n && e < lim && is_num(v.at(e))) e++;
    if (e == lim && e < n) return false;
    return (e == n || v.at(e) == ',') && parse_int_v(v, i, e, d);
}

// the "inside an item" state at the first byte a of this lane's `per` bytes
__device__ __forceinline__ bool rl_lane_inside(const RlView& v, int64_t a, int per) {
    const int lane = lane_id();
    int64_t last = -1;   // this lane's last parenthesis (2 * position + open), -1: none
    for (int64_t i = a; i < a + per && i < v.n; i++) {
        const uint8_t c = v.at(i);
        if (c == '(' || c == ')') last = 2 * i + (c == '(');
    }
    int64_t ex = __shfl_up(last, 1, 64);
    if (lane == 0) ex = -1;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {   // exclusive max-scan over the lanes before
        const int64_t o = __shfl_up(ex, d, 64);
        if (lane >= d && o > ex) ex = o;
    }
    // before the tile: the last parenthesis among its RL_BEHIND preceding bytes
    const int64_t b = v.t0 - RL_BEHIND + (lane & (RL_BEHIND - 1));
    const bool par = lane < RL_BEHIND && b >= 0 && (v.at(b) == '(' || v.at(b) == ')');
    const unsigned long long pm = __ballot(par);
    bool tile_in = false;
    if (pm) tile_in = v.at(v.t0 - RL_BEHIND + (63 - __clzll((long long)pm))) == '(';
    return ex >= 0 ? (ex & 1) != 0 : tile_in;
}

struct RlLane {
    int64_t cnt, dsum, lsum, lastlen;   // items starting in the lane, their deltas, lengths, the last length (-1)
};

// walk the lane's bytes: item starts (in order) to f(i, d, l); byte-class errors to err
template <typename F>
__device__ __forceinline__ RlLane rl_lane(const RlView& v, int64_t a, bool inside, int32_t* err, F&& f) {
    RlLane r{0, 0, 0, -1};
    bool bad = false;
    uint8_t prev = a > 0 ? v.at(a - 1) : (uint8_t)',';
    for (int64_t i = a; i < a + RL_LANE && i < v.n; i++) {
        const uint8_t c = v.at(i);
        bool start = false;
        if (c == '(') { start = true; inside = true; }
        else if (c == ')') { inside = false; }
        else if (!inside) {
            if (is_num(c)) start = !(i > 0 && is_num(prev));
            else if (c != ',') bad = true;
        }
        if (start) {
            int64_t d = 0, l = 1;
            if (!rl_item(v, i, &d, &l)) bad = true;
            f(i, d, l, r);
            r.cnt++;
            r.dsum += d;
            r.lsum += l;
            r.lastlen = l;
        }
        prev = c;
    }
    if (bad && err) atomicOr(err, 1);
    return r;
}

// One launch set parses both run lines: tiles [0, j0.ntiles) are line 0's, the rest line 1's.
struct RlJob {
    const uint8_t* s;
    int64_t n, ntiles;
    int64_t* tsum;      // 4 per tile: pass-1 summaries, then their exclusive prefixes
    int32_t* start;
    int32_t* len;
    int64_t* cum;
    int64_t* d_count;   // [0] items, [1] total length
};
__device__ __forceinline__ const RlJob& rl_job(const RlJob& j0, const RlJob& j1, int64_t& t) {
    if (t < j0.ntiles) return j0;
    t -= j0.ntiles;
    return j1;
}

// pass 1: per tile (count, delta sum, length sum, last length) -> tsum[4 * t]
__global__ __launch_bounds__(256) void k_rl_tiles(RlJob j0, RlJob j1, int32_t* __restrict__ err) {
    __shared__ uint8_t stage[4][RL_STAGE];
    int64_t t = (int64_t)blockIdx.x * 4 + wave_in_block();
    if (t >= j0.ntiles + j1.ntiles) return;
    const RlJob& J = rl_job(j0, j1, t);
    const int64_t t0 = t * RL_TILE, n = J.n;
    const int lane = lane_id();
    const RlView v = rl_stage<RL_TILE>(J.s, n, t0, stage[wave_in_block()]);
    const int64_t a = t0 + (int64_t)lane * RL_LANE;
    const bool inside = rl_lane_inside(v, a, RL_LANE);
    const RlLane r = rl_lane(v, a, inside, err, [](int64_t, int64_t, int64_t, const RlLane&) {});
    const int64_t c = wave_sum(r.cnt), d = wave_sum(r.dsum), l = wave_sum(r.lsum);
    const unsigned long long hm = __ballot(r.cnt > 0);
    const int64_t last = hm ? __shfl(r.lastlen, 63 - __clzll((long long)hm), 64) : -1;
    int64_t* tsum = J.tsum;
    if (lane == 0) { tsum[4 * t] = c; tsum[4 * t + 1] = d; tsum[4 * t + 2] = l; tsum[4 * t + 3] = last; }
    // the lane's own totals for the write pass (after the 4 * ntiles summaries)
    int64_t* ld = tsum + 4 * J.ntiles + (t * 64 + lane) * 4;
    ld[0] = r.cnt; ld[1] = r.dsum; ld[2] = r.lsum; ld[3] = r.lastlen;
}

// pass 2 (one block): exclusive prefix over tiles of (count, deltas, lengths) and the last item
// length before each tile (-1: none); the totals -> d_count[0..1]
constexpr int RL_SCAN_T = 256;   // (a 1024-thread block waits for a whole CU beside a running strip)
constexpr int RL_SCAN_B = 8;     // tile summaries per batch of loads
__device__ __forceinline__ int64_t i64_of(int lo, int hi) { return (int64_t)(((uint64_t)(uint32_t)hi << 32) | (uint32_t)lo); }
__global__ __launch_bounds__(RL_SCAN_T) void k_rl_scan(RlJob j0, RlJob j1) {   // block b: line b
    constexpr int NW = RL_SCAN_T / 64;
    __shared__ int64_t wc[NW], wd[NW], wl[NW], wlast[NW];
    const RlJob& J = blockIdx.x == 0 ? j0 : j1;
    const int64_t ntiles = J.ntiles;
    int64_t* tsum = J.tsum;
    int64_t* d_count = J.d_count;
    if (ntiles <= 0) {
        if (threadIdx.x == 0 && d_count) { d_count[0] = 0; d_count[1] = 0; }
        return;
    }
    const int tid = (int)threadIdx.x, lane = lane_id(), w = wave_in_block();
    const int64_t per = (ntiles + RL_SCAN_T - 1) / RL_SCAN_T, b0 = tid * per;
    const int64_t b1 = b0 + per < ntiles ? b0 + per : ntiles;
    // (RL_SCAN_B tiles' summaries loaded together: one tile at a time made this single-block pass
    // a chain of dependent HBM round trips, ~30 us on the chr1 reconstruction's critical path)
    int64_t c = 0, d = 0, l = 0, last = -1;
    for (int64_t t0 = b0; t0 < b1; t0 += RL_SCAN_B) {
        int4 q[RL_SCAN_B][2];
#pragma unroll
        for (int u = 0; u < RL_SCAN_B; u++)
            if (t0 + u < b1) {
                const int4* p4 = reinterpret_cast<const int4*>(tsum + 4 * (t0 + u));
                q[u][0] = p4[0];
                q[u][1] = p4[1];
            }
#pragma unroll
        for (int u = 0; u < RL_SCAN_B; u++)
            if (t0 + u < b1) {
                c += i64_of(q[u][0].x, q[u][0].y); d += i64_of(q[u][0].z, q[u][0].w); l += i64_of(q[u][1].x, q[u][1].y);
                const int64_t tl = i64_of(q[u][1].z, q[u][1].w);
                if (tl >= 0) last = tl;
            }
    }
    int64_t ic = c, id = d, il = l, ilast = last;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const int64_t xc = __shfl_up(ic, o, 64), xd = __shfl_up(id, o, 64), xl = __shfl_up(il, o, 64),
                      xlast = __shfl_up(ilast, o, 64);
        if (lane >= o) { ic += xc; id += xd; il += xl; if (ilast < 0) ilast = xlast; }
    }
    if (lane == 63) { wc[w] = ic; wd[w] = id; wl[w] = il; wlast[w] = ilast; }
    __syncthreads();
    int64_t pc = 0, pd = 0, pl = 0, plast = -1;
    for (int i = 0; i < w; i++) { pc += wc[i]; pd += wd[i]; pl += wl[i]; if (wlast[i] >= 0) plast = wlast[i]; }
    int64_t ec = pc + ic - c, ed = pd + id - d, el = pl + il - l;
    int64_t elast = __shfl_up(ilast, 1, 64);
    if (lane == 0 || elast < 0) elast = lane == 0 ? plast : (elast < 0 ? plast : elast);
    for (int64_t t0 = b0; t0 < b1; t0 += RL_SCAN_B) {
        int4 q[RL_SCAN_B][2];
#pragma unroll
        for (int u = 0; u < RL_SCAN_B; u++)
            if (t0 + u < b1) {
                const int4* p4 = reinterpret_cast<const int4*>(tsum + 4 * (t0 + u));
                q[u][0] = p4[0];
                q[u][1] = p4[1];
            }
#pragma unroll
        for (int u = 0; u < RL_SCAN_B; u++)
            if (t0 + u < b1) {
                const int64_t t = t0 + u;
                const int64_t tc = i64_of(q[u][0].x, q[u][0].y), td = i64_of(q[u][0].z, q[u][0].w);
                const int64_t tl = i64_of(q[u][1].x, q[u][1].y), tlast = i64_of(q[u][1].z, q[u][1].w);
                tsum[4 * t] = ec; tsum[4 * t + 1] = ed; tsum[4 * t + 2] = el; tsum[4 * t + 3] = elast;
                ec += tc; ed += td; el += tl;
                if (tlast >= 0) elast = tlast;
            }
    }
    if (tid == RL_SCAN_T - 1 && d_count) { d_count[0] = ec; d_count[1] = el; }
}

// pass 3: every item's start (running sum of deltas), length and the exclusive prefix of lengths;
// starts must be >= 0, ascending and disjoint, and end within int32 (k_run_finish's checks)
__global__ __launch_bounds__(256) void k_rl_write(RlJob j0, RlJob j1, int32_t* __restrict__ err) {
    __shared__ uint8_t stage[4][RL_STAGE];
    int64_t t = (int64_t)blockIdx.x * 4 + wave_in_block();
    if (t >= j0.ntiles + j1.ntiles) return;
    const RlJob& J = rl_job(j0, j1, t);
    const int64_t t0 = t * RL_TILE, n = J.n;
    const int64_t* tsum = J.tsum;
    int32_t* start = J.start;
    int32_t* len = J.len;
    int64_t* cum = J.cum;
    const int lane = lane_id();
    const RlView v = rl_stage<RL_TILE>(J.s, n, t0, stage[wave_in_block()]);
    const int64_t a = t0 + (int64_t)lane * RL_LANE;
    const bool inside = rl_lane_inside(v, a, RL_LANE);
    // the lane's totals (pass 1 kept them), then its exclusive prefixes over the wave
    const int64_t* ld = tsum + 4 * J.ntiles + (t * 64 + lane) * 4;
    const RlLane tot{ld[0], ld[1], ld[2], ld[3]};
    const int64_t ic = wave_incl_add(tot.cnt), id = wave_incl_add(tot.dsum), il = wave_incl_add(tot.lsum);
    // the last item length before this lane (in earlier lanes, else before the tile)
    const unsigned long long hm = __ballot(tot.cnt > 0) & ((1ull << lane) - 1ull);
    const int64_t prevlen = hm ? __shfl(tot.lastlen, 63 - __clzll((long long)hm), 64) : tsum[4 * t + 3];
    const int64_t rank0 = tsum[4 * t] + ic - tot.cnt;
    int64_t run_start = tsum[4 * t + 1] + id - tot.dsum;   // start of the last item before this lane's first
    int64_t run_cum = tsum[4 * t + 2] + il - tot.lsum;
    int64_t prev_end = rank0 > 0 ? run_start + (prevlen >= 0 ? prevlen : 0) : INT64_MIN;
    bool bad = false;
    rl_lane(v, a, inside, nullptr, [&](int64_t, int64_t d, int64_t l, const RlLane& r) {
        const int64_t rank = rank0 + r.cnt;
        const int64_t st = run_start + d;
        if (st < 0 || st + l > INT32_MAX || (rank > 0 && st < prev_end)) bad = true;
        start[rank] = (int32_t)st;
        len[rank] = (int32_t)l;
        cum[rank] = run_cum;
        run_start = st;
        run_cum += l;
        prev_end = st + l;
    });
    if (bad) atomicOr(err, 1);
}

// starts = inclusive prefix of deltas (exclusive scan + own delta); runs must be ascending & disjoint.
// Also the run lengths as int64 for the N-count prefix, 0 past the *d_nr parsed runs (the scans run
// to the capacity, so the host never waits for the count).
__global__ void k_run_finish(const int64_t* __restrict__ dex, const int64_t* __restrict__ dlt, const int32_t* __restrict__ len,
                             int64_t cap, const int64_t* __restrict__ d_nr, int32_t* __restrict__ start,
                             int64_t* __restrict__ len64, int32_t* __restrict__ err) {
    const int64_t nr = *d_nr;
    for (int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; r < cap; r += (int64_t)gridDim.x * blockDim.x) {
        if (r >= nr) { len64[r] = 0; continue; }
        const int64_t st = dex[r] + dlt[r];
        const int64_t pst = r ? dex[r - 1] + dlt[r - 1] : INT64_MIN;
        const int64_t pend = r ? pst + len[r - 1] : 0;
        // (the formatter keeps run ends in int32: a run must also END within int32)
        if (st < 0 || st + (int64_t)len[r] > INT32_MAX || (r && st < pend)) atomicOr(err, 1);
        start[r] = (int32_t)st;
        len64[r] = len[r];
    }
}

// the last N run must end within the sequence: decoded length (*d_D) + N count (d_ncnt[1])
__global__ void k_n_check(const int32_t* __restrict__ ns, const int32_t* __restrict__ nl, const int64_t* __restrict__ d_ncnt,
                          const int64_t* __restrict__ d_D, int32_t* __restrict__ err) {
    const int64_t n = d_ncnt[0];
    if (threadIdx.x == 0 && n > 0 && (int64_t)ns[n - 1] + nl[n - 1] > *d_D + d_ncnt[1]) atomicOr(err, 4);
}

// ---------------------------------------------------------------------------------------------
// record line
// ---------------------------------------------------------------------------------------------
// per byte: output contribution (literal 1, token l, else 0) and token delta (tokens only)
__global__ void k_tok_parse(const uint8_t* __restrict__ s, int64_t n, const int64_t* __restrict__ lp,
                            int64_t* __restrict__ contrib, int64_t* __restrict__ dlt, int32_t* __restrict__ err) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        const uint8_t c = s[i];
        const bool inside = lp[i] >= 0 && s[lp[i]] == '(';
        int64_t cb = 0, d = 0;
        if (c == '(') {
            int64_t comma = -1, close = -1;
            for (int64_t q = i + 1; q < n && q < i + 32; q++) {
                if (s[q] == ',' && comma < 0) comma = q;
                if (s[q] == ')') { close = q; break; }
                if (s[q] == '(') break;
            }
            int64_t l = 0;
            if (!(comma > 0 && close > comma && parse_int(s, n, i + 1, comma, &d) && parse_int(s, n, comma + 1, close, &l)) || l < 0)
                atomicOr(err, 1);
            cb = l;
        } else if (c == ')') {
            cb = inside ? 0 : 1;             // a ')' outside a token is a literal (decompression.cpp:231-234)
        } else if (!inside) {
            cb = 1;
        }
        contrib[i] = cb;
        dlt[i] = d;
    }
}

// absolute p = running sum of deltas over tokens (decompression.cpp:220-222); range check :223
__global__ void k_tok_check(const uint8_t* __restrict__ s, int64_t n, const int64_t* __restrict__ dsum,
                            const int64_t* __restrict__ dlt, const int64_t* __restrict__ contrib,
                            const int64_t* __restrict__ d_nref, int32_t* __restrict__ err) {
    const int64_t nref = *d_nref;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        if (s[i] != '(') continue;
        const int64_t p = dsum[i] + dlt[i];
        if (p < 0 || p + contrib[i] > nref) atomicOr(err, 2);
    }
}

constexpr int WPB = 4;
// 16 bytes from any byte address: one global_load_dwordx4 (gfx950 runs in unaligned access mode;
// SCCG_UNALIGNED_LD=0: five dword loads combined with v_alignbyte, as before round 6)
#ifndef SCCG_UNALIGNED_LD
#define SCCG_UNALIGNED_LD 1
#endif
__device__ __forceinline__ uint4 load16u(const uint8_t* __restrict__ p) {
    uint4 v;
    if (SCCG_UNALIGNED_LD) {
        __builtin_memcpy(&v, p, 16);
    } else {
        const uint32_t* sa = reinterpret_cast<const uint32_t*>((uintptr_t)p & ~(uintptr_t)3);
        const unsigned sh = (unsigned)((uintptr_t)p & 3);
        uint32_t w[5];
#pragma unroll
        for (int i = 0; i < 5; i++) w[i] = sa[i];
        v = make_uint4(__builtin_amdgcn_alignbyte(w[1], w[0], sh), __builtin_amdgcn_alignbyte(w[2], w[1], sh),
                       __builtin_amdgcn_alignbyte(w[3], w[2], sh), __builtin_amdgcn_alignbyte(w[4], w[3], sh));
    }
    return v;
}
// dst[0, l) = src[0, l) by one wave: bytes up to dst's next 16-byte boundary and after its last one
// one per lane, the rest 16 bytes per lane as aligned stores of (unaligned) 16-byte source loads.
// The source may be read up to 19 bytes past src + l (the reference buffers carry 64 bytes of slack).
#ifndef WC_DEPTH
#define WC_DEPTH 2
#endif
__device__ __forceinline__ void wave_copy_body(uint4* __restrict__ d, const uint8_t* __restrict__ s0, int64_t nb, int64_t from,
                                               int lane);
__device__ __forceinline__ int64_t readlane64(int64_t v, int l) {
    const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int32_t)v, l);
    const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int32_t)(v >> 32), l);
    return (int64_t)(((uint64_t)hi << 32) | lo);
}
__device__ __forceinline__ void wave_copy(uint8_t* __restrict__ dst, const uint8_t* __restrict__ src, int64_t l, int lane) {
    const int64_t h = ((16 - ((uintptr_t)dst & 15)) & 15) < l ? ((16 - ((uintptr_t)dst & 15)) & 15) : l;
    const int64_t nb = (l - h) >> 4;
    const int64_t t0 = h + (nb << 4);
    if (lane < h) dst[lane] = src[lane];
    if (lane < l - t0) dst[t0 + lane] = src[t0 + lane];
    wave_copy_body(reinterpret_cast<uint4*>(dst + h), src + h, nb, 0, lane);
}

// 16-byte chunks [from, nb) of d = s0 (d 16-byte aligned)
__device__ __forceinline__ void wave_copy_body(uint4* __restrict__ d, const uint8_t* __restrict__ s0, int64_t nb, int64_t from,
                                               int lane) {
    // WC_DEPTH KiB of loads in flight per wave before the stores (one 1 KiB step at a time left the
    // fill bound by the bytes in flight: ~3 TB/s)
    for (int64_t c0 = from + lane; c0 < nb; c0 += 64 * WC_DEPTH) {
        uint4 v[WC_DEPTH];
#pragma unroll
        for (int u = 0; u < WC_DEPTH; u++) {
            const int64_t c = c0 + 64 * u;
            if (c < nb) v[u] = load16u(s0 + 16 * c);
        }
#pragma unroll
        for (int u = 0; u < WC_DEPTH; u++) {
            const int64_t c = c0 + 64 * u;
            if (c < nb) d[c] = v[u];
        }
    }
}

__global__ __launch_bounds__(SCCG_BLOCK) void k_tok_fill(const uint8_t* __restrict__ s, int64_t n,
                                                         const int64_t* __restrict__ lp, const int64_t* __restrict__ off,
                                                         const int64_t* __restrict__ dsum, const int64_t* __restrict__ dlt,
                                                         const int64_t* __restrict__ contrib, const uint8_t* __restrict__ R,
                                                         uint8_t* __restrict__ dec) {
    // one wave per 64-byte stretch of the record line; tokens are copied by the whole wave
    const int64_t base = ((int64_t)blockIdx.x * WPB + wave_in_block()) * 64;
    if (base >= n) return;
    const int lane = lane_id();
    const int64_t i = base + lane;
    bool tok = false;
    int64_t p = 0, l = 0, o = 0;
    if (i < n) {
        const uint8_t c = s[i];
        const bool inside = lp[i] >= 0 && s[lp[i]] == '(';
        if (c == '(') {
            tok = true;
            p = dsum[i] + dlt[i];
            l = contrib[i];
            o = off[i];
        } else if (!inside) {
            dec[off[i]] = c;   // literals, a stray ')' included
        }
    }
    unsigned long long tm = __ballot(tok);
    while (tm) {
        const int j = __ffsll((long long)tm) - 1;
        tm &= tm - 1;
        const int64_t pj = __shfl(p, j), lj = __shfl(l, j), oj = __shfl(o, j);
        wave_copy(dec + oj, R + pj, lj, lane);
    }
}

// ---------------------------------------------------------------------------------------------
// record line, per 64-byte block (the usual path).  A token "(dp,l)" is at most 25 bytes, so the
// "inside a token" state at a block's first byte follows from the last parenthesis before it (the
// lanes before it in the 1 KiB tile, else the 32 bytes before the tile; rl_lane_inside).  Pass 1
// stores per block its state and its sums of output bytes (literal 1, token l) and token deltas;
// two exclusive scans over the blocks give every block's output offset and running p; the fill
// recomputes a block's bytes from those (decompression.cpp:210-236), with the range check of
// :223-229 (d_err bit 2) in the same pass.  (The per-byte arrays of the scan-based path -- last
// parenthesis, contribution, delta, their prefix sums: 40 B per record byte -- are gone.)
// ---------------------------------------------------------------------------------------------
constexpr int TK_B = 64;   // record bytes per block (one lane in pass 1, one wave in the fill)

__global__ __launch_bounds__(256) void k_tok_blocks(const uint8_t* __restrict__ s, int64_t n, int64_t* __restrict__ bin,
                                                    int64_t* __restrict__ bcontrib, int64_t* __restrict__ bdelta,
                                                    int32_t* __restrict__ err, int64_t* __restrict__ btok) {
    // one wave per 1 KiB tile (16 bytes per lane, staged in LDS); 4 lanes make one 64-byte block
    constexpr int TL = 16, TT = 64 * TL;
    __shared__ uint8_t stage[4][RL_BEHIND + TT + RL_AHEAD];
    const int64_t t = (int64_t)blockIdx.x * 4 + wave_in_block();
    const int64_t t0 = t * TT;
    if (t0 >= n) return;
    const int lane = lane_id();
    const RlView v = rl_stage<TT>(s, n, t0, stage[wave_in_block()]);
    const int64_t a = t0 + (int64_t)lane * TL;
    bool inside = rl_lane_inside(v, a, TL);
    const bool in0 = inside;
    int64_t cs = 0, ds = 0, tk = 0;
    bool bad = false;
    for (int64_t i = a; i < a + TL && i < n; i++) {
        const uint8_t c = v.at(i);
        if (c == '(') {
            int64_t comma = -1, close = -1, d = 0, l = 0;
            for (int64_t q = i + 1; q < n && q < i + 32; q++) {
                const uint8_t cq = v.at(q);
                if (cq == ',' && comma < 0) comma = q;
                if (cq == ')') { close = q; break; }
                if (cq == '(') break;
            }
            if (!(comma > 0 && close > comma && parse_int_v(v, i + 1, comma, &d) && parse_int_v(v, comma + 1, close, &l)) ||
                l < 0)
                bad = true;
            else
                tk++;
            cs += l;
            ds += d;
            inside = true;
        } else if (c == ')') {
            cs += inside ? 0 : 1;   // a ')' outside a token is a literal (decompression.cpp:231-234)
            inside = false;
        } else if (!inside) {
            cs += 1;
        }
    }
    if (bad) atomicOr(err, 1);
    cs += __shfl_xor(cs, 1, 64);
    cs += __shfl_xor(cs, 2, 64);
    ds += __shfl_xor(ds, 1, 64);
    ds += __shfl_xor(ds, 2, 64);
    tk += __shfl_xor(tk, 1, 64);
    tk += __shfl_xor(tk, 2, 64);
    static_assert(4 * TL == TK_B, "four lanes per block");
    const int64_t b = t * (TT / TK_B) + (lane >> 2);
    if ((lane & 3) == 0 && b * TK_B < n) {
        bin[b] = in0;
        bcontrib[b] = cs;
        bdelta[b] = ds;
        if (btok) btok[b] = tk;
    }
}

// one wave per block: literals and token copies into dec at the block's offsets; tokens beyond
// the reference (p < 0 or p + l > |R'|, decompression.cpp:223-229) set d_err bit 2 and copy nothing.
// WRITE = false: the range check alone (no dec; a size query or an early error must report
// SCCG_E_RANGE exactly as the full decode would)
template <bool WRITE>
__global__ __launch_bounds__(SCCG_BLOCK) void k_tok_fill2(const uint8_t* __restrict__ s, int64_t n,
                                                          const int64_t* __restrict__ bin, const int64_t* __restrict__ boff,
                                                          const int64_t* __restrict__ bdsum, const int64_t* __restrict__ d_nref,
                                                          const uint8_t* __restrict__ R, uint8_t* __restrict__ dec,
                                                          int32_t* __restrict__ err, int64_t dcap) {
    __shared__ uint8_t stg[WPB][2 * TK_B];
    const int64_t b = (int64_t)blockIdx.x * WPB + wave_in_block();
    const int64_t base = b * TK_B;
    if (base >= n) return;
    const int lane = lane_id();
    const int64_t i = base + lane;
    // the block's 64 bytes and the 64 after them (a token starting in the block ends within 32) in
    // LDS: the token parses below read LDS, not one dependent HBM byte after the other
    uint8_t* st = stg[wave_in_block()];
    const uint8_t c = i < n ? s[i] : (uint8_t)',';
    st[lane] = c;
    st[TK_B + lane] = i + TK_B < n ? s[i + TK_B] : (uint8_t)0;
    wave_sync();
    const RlView v{st - RL_BEHIND, base, n, TK_B};   // v.at(q) = st[q - base]
    const bool par = i < n && (c == '(' || c == ')');
    // the last parenthesis strictly before this byte inside the block, else the block's state
    const unsigned long long pm = __ballot(par) & ((1ull << lane) - 1ull);
    const bool inside = pm ? st[63 - __clzll((long long)pm)] == '(' : bin[b] != 0;
    int64_t contrib = 0, d = 0;
    bool tok = false;
    if (i < n) {
        if (c == '(') {
            int64_t comma = -1, close = -1, l = 0;
            for (int64_t q = i + 1; q < n && q < i + 32; q++) {
                const uint8_t cq = v.at(q);
                if (cq == ',' && comma < 0) comma = q;
                if (cq == ')') { close = q; break; }
                if (cq == '(') break;
            }
            if (comma > 0 && close > comma && parse_int_v(v, i + 1, comma, &d) && parse_int_v(v, comma + 1, close, &l) && l >= 0) {
                tok = true;
                contrib = l;
            }
        } else if (c == ')') {
            contrib = inside ? 0 : 1;
        } else if (!inside) {
            contrib = 1;
        }
    }
    const int64_t o = boff[b] + wave_incl_add(contrib) - contrib;
    const int64_t p = bdsum[b] + wave_incl_add(d);   // running p, this token included
    const int64_t nref = *d_nref;
    if (tok && (p < 0 || p + contrib > nref)) {
        atomicOr(err, 2);
        tok = false;
    }
    if (!WRITE) return;
    // (dcap: dec's capacity -- a fill queued before the decoded length is known writes nothing past
    // it; only a call that then fails its output-capacity check can reach it)
    if (!tok && contrib == 1 && c != '(' && o < dcap) dec[o] = c;   // literals, a stray ')' included
    unsigned long long tm = __ballot(tok);
    while (tm) {
        const int j = __ffsll((long long)tm) - 1;   // (wave-uniform: the token's fields by readlane)
        tm &= tm - 1;
        const int64_t pj = readlane64(p, j), oj = readlane64(o, j);
        int64_t lj = readlane64(contrib, j);
        if (lj > dcap - oj) lj = dcap - oj > 0 ? dcap - oj : 0;
        wave_copy(dec + oj, R + pj, lj, lane);
    }
}

// Token table of the fused reconstruction (opt-in, SCCG_DC_FUSED=1): instead of copying bytes into a decoded
// buffer that the formatter reads back (k_tok_fill2), one wave per 64-byte block writes each token's
// decoded offset o, absolute reference position p, length l and the record offset r right after its
// ')' (decompression.cpp:210-236).  Entry 0 is a sentinel (0, 0, 0, 0) for the literals before the
// first token; token j of the line is entry 1 + j.  Decoded byte x then lies in entry t = the last
// with o_t <= x: it is R'[p_t + x - o_t] when x < o_t + l_t, else the literal rec[r_t + x - o_t - l_t]
// (between a token's ')' and the next '(' every byte is a literal, :231-236).  Needs no R', so it
// runs beside the reference strip; the range check (:223-229) is k_tok_range, after the strip.
__global__ __launch_bounds__(SCCG_BLOCK) void k_tok_emit(const uint8_t* __restrict__ s, int64_t n,
                                                         const int64_t* __restrict__ bin, const int64_t* __restrict__ boff,
                                                         const int64_t* __restrict__ bdsum, const int64_t* __restrict__ btoff,
                                                         DcTokTab tk) {
    __shared__ uint8_t stg[WPB][2 * TK_B];
    const int64_t b = (int64_t)blockIdx.x * WPB + wave_in_block();
    const int64_t base = b * TK_B;
    if (base >= n) return;
    const int lane = lane_id();
    const int64_t i = base + lane;
    uint8_t* st = stg[wave_in_block()];
    const uint8_t c = i < n ? s[i] : (uint8_t)',';
    st[lane] = c;
    st[TK_B + lane] = i + TK_B < n ? s[i + TK_B] : (uint8_t)0;
    wave_sync();
    const RlView v{st - RL_BEHIND, base, n, TK_B};
    const bool par = i < n && (c == '(' || c == ')');
    const unsigned long long pm = __ballot(par) & ((1ull << lane) - 1ull);
    const bool inside = pm ? st[63 - __clzll((long long)pm)] == '(' : bin[b] != 0;
    int64_t contrib = 0, d = 0, close = -1;
    bool tok = false;
    if (i < n) {
        if (c == '(') {
            int64_t comma = -1, l = 0;
            for (int64_t q = i + 1; q < n && q < i + 32; q++) {
                const uint8_t cq = v.at(q);
                if (cq == ',' && comma < 0) comma = q;
                if (cq == ')') { close = q; break; }
                if (cq == '(') break;
            }
            if (comma > 0 && close > comma && parse_int_v(v, i + 1, comma, &d) && parse_int_v(v, comma + 1, close, &l) && l >= 0) {
                tok = true;
                contrib = l;
            }
        } else if (c == ')') {
            contrib = inside ? 0 : 1;
        } else if (!inside) {
            contrib = 1;
        }
    }
    const int64_t o = boff[b] + wave_incl_add(contrib) - contrib;
    const int64_t p = bdsum[b] + wave_incl_add(d);   // running p, this token included
    const unsigned long long tm = __ballot(tok);
    if (tok) {
        const int64_t e = 1 + btoff[b] + __popcll(tm & ((1ull << lane) - 1ull));
        tk.o[e] = o;
        tk.p[e] = p;
        tk.l[e] = contrib;
        tk.r[e] = close + 1;
    }
    if (b == 0 && lane == 0) { tk.o[0] = 0; tk.p[0] = 0; tk.l[0] = 0; tk.r[0] = 0; }
}

// d_err bit 2 for a token beyond the reference (p < 0 or p + l > |R'|, decompression.cpp:223-229)
__global__ void k_tok_range(DcTokTab tk, const int64_t* __restrict__ d_ntok, const int64_t* __restrict__ d_nref,
                            int32_t* __restrict__ err) {
    const int64_t nt = *d_ntok, nref = *d_nref;
    bool bad = false;
    for (int64_t t = 1 + (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t <= nt; t += (int64_t)gridDim.x * blockDim.x) {
        const int64_t p = tk.p[t], l = tk.l[t];
        if (p < 0 || p + l > nref) bad = true;
    }
    if (bad) atomicOr(err, 2);
}

// ---------------------------------------------------------------------------------------------
// output: header '\n' then result wrapped at 50 columns + final '\n'
// ---------------------------------------------------------------------------------------------
__device__ __forceinline__ int64_t first_run_ending_after(const int32_t* st, const int32_t* ln, int64_t nr, int64_t j,
                                                          int64_t a = 0) {
    int64_t b = nr;   // first r >= a with st[r] + ln[r] > j (runs sorted and disjoint)
    while (a < b) {
        const int64_t m = (a + b) >> 1;
        if ((int64_t)st[m] + ln[m] > j) b = m; else a = m + 1;
    }
    return a;
}

// A block owns FSPAN consecutive sequence positions.  Their decoded bytes (one contiguous range
// of dec, N positions excluded) are loaded into LDS with stride-1 reads, every thread formats FPER
// positions into the block's LDS copy of its output range (N runs, lowercase runs, a '\n' after
// every 50th base but the last), and the block stores that range with stride-1 writes.  (A
// thread-per-64-positions writer straight to HBM, lanes 64 bytes apart, took 4.6 ms for a
// chr1-sized FASTA.)
constexpr int FPER = 16, FSPAN = 256 * FPER;
// N positions before j (j inside an N run: those of the run before j included), given
// r = first_run_ending_after(ns, nl, nn, j)
__device__ __forceinline__ int64_t n_before_at(const int32_t* ns, const int32_t* nl, const int64_t* ncum, int64_t nn,
                                               int64_t r, int64_t j) {
    if (r < nn) return ncum[r] + (ns[r] <= j ? j - ns[r] : 0);
    return nn ? ncum[nn - 1] + nl[nn - 1] : 0;
}

// Span boundaries J_b = min(b * FSPAN, nres), b = 0..nspan: the first N run and the first
// lowercase run ending after J_b, and J_b minus the N positions before it (the decoded-byte offset
// of J_b).  One thread per (boundary, run list), all independent: the dependent binary-search loads
// overlap across the grid instead of sitting at the head of every format block (a per-block search
// chain of ~36 loads x 30 block generations took 0.79 ms of a chr1 reconstruction).
__global__ void k_span_index(int64_t nres, int64_t nspan, const int32_t* __restrict__ ns, const int32_t* __restrict__ nl,
                             const int64_t* __restrict__ ncum, int64_t nn, const int32_t* __restrict__ ls,
                             const int32_t* __restrict__ ll, int64_t nlr, int64_t* __restrict__ tab) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < 2 * (nspan + 1); i += (int64_t)gridDim.x * blockDim.x) {
        const int64_t b = i >> 1;
        const int64_t J = b * FSPAN < nres ? b * FSPAN : nres;
        if (i & 1) {
            tab[3 * b + 2] = first_run_ending_after(ls, ll, nlr, J);
        } else {
            const int64_t r = first_run_ending_after(ns, nl, nn, J);
            tab[3 * b + 0] = J - n_before_at(ns, nl, ncum, nn, r, J);
            tab[3 * b + 1] = r;
        }
    }
}

// Run-list views for format_positions: starts, ends and (N runs) the N count before each run,
// read from the span's LDS copies or from the global lists.
struct LdsRuns {
    const int32_t* s;
    const int32_t* e;
    const int64_t* b;
    __device__ int64_t st(int64_t r) const { return s[r]; }
    __device__ int64_t en(int64_t r) const { return e[r]; }
    __device__ int64_t nb(int64_t r) const { return b[r]; }
};
struct GlobalRuns {
    const int32_t* s;
    const int32_t* l;
    const int64_t* b;
    __device__ int64_t st(int64_t r) const { return s[r]; }
    __device__ int64_t en(int64_t r) const { return (int64_t)s[r] + l[r]; }
    __device__ int64_t nb(int64_t r) const { return b[r]; }
};

// Formats positions [j0, j0 + FPER) of a span (j < J1) into sout; rn / rl enter as the first
// N / lowercase run ending after j0 (runs past the views' counts: none left, ntot N before).
template <typename V>
__device__ __forceinline__ void format_positions(int64_t j0, int64_t J1, int64_t nres, int64_t O0, int64_t dbase,
                                                 const uint8_t* sdec, uint8_t* sout, V N, int64_t nn, int64_t ntot, V L,
                                                 int64_t nlr, int64_t rn, int64_t rl) {
    int64_t n_s = INT64_MAX, n_e = INT64_MAX, n_b = ntot, l_s = INT64_MAX, l_e = INT64_MAX;
    if (rn < nn) { n_s = N.st(rn); n_e = N.en(rn); n_b = N.nb(rn); }
    if (rl < nlr) { l_s = L.st(rl); l_e = L.en(rl); }
    // output offset of j = j + j / 50 - O0, kept as a running column (no 64-bit division per base)
    int64_t o = j0 + j0 / 50 - O0;
    int col = (int)(j0 % 50);
    const int64_t je = j0 + FPER < J1 ? j0 + FPER : J1;
    for (int64_t j = j0; j < je; j++) {
        while (j >= n_e) {
            rn++;
            if (rn < nn) { n_s = N.st(rn); n_e = N.en(rn); n_b = N.nb(rn); }
            else { n_s = n_e = INT64_MAX; n_b = ntot; }
        }
        while (j >= l_e) {
            rl++;
            if (rl < nlr) { l_s = L.st(rl); l_e = L.en(rl); }
            else l_s = l_e = INT64_MAX;
        }
        uint8_t c = j >= n_s ? (uint8_t)'N' : sdec[j - n_b - dbase];
        if (j >= l_s) c = c_tolower(c);
        sout[o++] = c;
        if (++col == 50) {
            col = 0;
            if (j != nres - 1) sout[o++] = '\n';
        }
    }
}

// first r in [a, b) with V::en(r) > j, ends ascending
template <typename V>
__device__ __forceinline__ int64_t first_end_after(const V& v, int64_t a, int64_t b, int64_t j) {
    while (a < b) {
        const int64_t m = (a + b) >> 1;
        if (v.en(m) > j) b = m; else a = m + 1;
    }
    return a;
}

// One block per span.  The span's decoded bytes (dword loads), and when they are few (<= FRUNS
// each, the usual case) the N and lowercase runs it touches, are staged in LDS in one round trip
// behind the span table; every thread then formats FPER positions from LDS only, and the block
// stores its output range with dword stores.  Spans with dense run alternation read the run
// lists from global memory instead.
constexpr int FRUNS = 384;
__global__ __launch_bounds__(256) void k_format_span(const uint8_t* __restrict__ dec, int64_t nres,
                                                     const int32_t* __restrict__ ns, const int32_t* __restrict__ nl,
                                                     const int64_t* __restrict__ ncum, int64_t nn,
                                                     const int32_t* __restrict__ ls, const int32_t* __restrict__ ll,
                                                     int64_t nlr, const int64_t* __restrict__ tab, uint8_t* __restrict__ out) {
    __shared__ uint32_t sdec_w[FSPAN / 4 + 2];
    __shared__ uint8_t sout[FSPAN + FSPAN / 50 + 8];
    __shared__ int32_t s_ns[FRUNS], s_ne[FRUNS], s_ls[FRUNS], s_le[FRUNS];
    __shared__ int64_t s_nb[FRUNS];
    __shared__ int64_t st[7];
    const int64_t b = blockIdx.x;
    const int64_t J0 = b * FSPAN;
    if (J0 >= nres) return;
    const int64_t J1 = J0 + FSPAN < nres ? J0 + FSPAN : nres;
    const int tid = threadIdx.x;
    if (tid < 6) st[tid] = tab[3 * b + tid];
    if (tid == 6) st[6] = nn ? ncum[nn - 1] + nl[nn - 1] : 0;
    __syncthreads();
    // the runs this span touches lie in [first(J0), first(J1)] (first = first run ending after)
    const int64_t d0 = st[0], dn = st[3] - d0;
    const int64_t n_lo = st[1], n_hi = st[4] < nn ? st[4] + 1 : nn;
    const int64_t l_lo = st[2], l_hi = st[5] < nlr ? st[5] + 1 : nlr;
    const int64_t ntot = st[6];
    const bool lds_runs = n_hi - n_lo <= FRUNS && l_hi - l_lo <= FRUNS;
    const int64_t a0 = d0 & ~(int64_t)3;
    const int64_t nw = (d0 + dn - a0 + 3) >> 2;
    const uint32_t* decw = reinterpret_cast<const uint32_t*>(dec + a0);
    for (int64_t i = tid; i < nw; i += 256) sdec_w[i] = decw[i];
    if (lds_runs) {
        for (int64_t r = n_lo + tid; r < n_hi; r += 256) {
            const int32_t x = ns[r];
            s_ns[r - n_lo] = x;
            s_ne[r - n_lo] = x + nl[r];
            s_nb[r - n_lo] = ncum[r];
        }
        for (int64_t r = l_lo + tid; r < l_hi; r += 256) {
            const int32_t x = ls[r];
            s_ls[r - l_lo] = x;
            s_le[r - l_lo] = x + ll[r];
        }
    }
    __syncthreads();
    const uint8_t* sdec = reinterpret_cast<const uint8_t*>(sdec_w);
    const int64_t O0 = J0 + J0 / 50;
    const int64_t jl = J1 - 1;
    const int64_t On = jl + jl / 50 + 1 + ((jl % 50 == 49 && jl != nres - 1) ? 1 : 0) - O0;
    const int64_t j0 = J0 + (int64_t)tid * FPER;
    if (j0 < J1) {
        if (lds_runs) {
            const int64_t cn = n_hi - n_lo, cl = l_hi - l_lo;
            const LdsRuns N{s_ns, s_ne, s_nb}, L{s_ls, s_le, nullptr};
            format_positions(j0, J1, nres, O0, a0, sdec, sout, N, cn, ntot, L, cl, first_end_after(N, 0, cn, j0),
                             first_end_after(L, 0, cl, j0));
        } else {
            const GlobalRuns N{ns, nl, ncum}, L{ls, ll, nullptr};
            format_positions(j0, J1, nres, O0, a0, sdec, sout, N, nn, ntot, L, nlr, first_end_after(N, n_lo, n_hi, j0),
                             first_end_after(L, l_lo, l_hi, j0));
        }
    }
    __syncthreads();
    // store [O0, O0 + On): bytes up to the first 4-byte boundary and after the last, dwords between
    uint8_t* o = out + O0;
    const int64_t h = ((4 - ((uintptr_t)o & 3)) & 3) < On ? ((4 - ((uintptr_t)o & 3)) & 3) : On;
    const int64_t nbw = (On - h) >> 2;
    const int64_t t0 = h + (nbw << 2);
    if (tid < h) o[tid] = sout[tid];
    if (tid < On - t0) o[t0 + tid] = sout[t0 + tid];
    uint32_t* ow = reinterpret_cast<uint32_t*>(o + h);
    for (int64_t i = tid; i < nbw; i += 256) {
        const uint8_t* q = sout + h + 4 * i;
        ow[i] = (uint32_t)q[0] | ((uint32_t)q[1] << 8) | ((uint32_t)q[2] << 16) | ((uint32_t)q[3] << 24);
    }
}

// ---------------------------------------------------------------------------------------------
// Output-centric formatter (the usual path).  A block owns OB = 4096 bytes of the OUTPUT, aligned
// to 16 bytes in memory; every thread builds 16 output bytes in registers and stores them with one
// 16-byte store (head and tail threads byte by byte).  Output byte o is the '\n' after a line when
// o % 51 == 50, else position j = o - o / 51; its byte is 'N' inside an N run, else the decoded
// byte at j minus the N positions before j, lowercased inside a lowercase run
// (decompression.cpp:241-274).  The block's decoded bytes and the runs it touches are staged in
// LDS (runs from the global lists when they are more than OFRUNS); a thread finds its first runs by
// binary search in LDS and then walks them.  (The position-centric k_format_span wrote each
// position's byte to LDS, 16 bytes apart per lane, and copied the line-broken range out again.)
// ---------------------------------------------------------------------------------------------
#ifndef SCCG_OFRUNS
#define SCCG_OFRUNS 384
#endif
constexpr int OPT = 16, OB = 256 * OPT, OFRUNS = SCCG_OFRUNS;   // (a block with more runs takes the global-runs path)
constexpr int TW = 5;   // k_out_index entries per block boundary
constexpr int FMT_U_DEFAULT = 4;   // (U = 1 / 2 / 4 on one box, chr1: 0.638-0.647 / 0.634-0.639 / 0.624-0.626 ms;
                                    //  round 6, U = 8: 42 KiB of LDS per block, 0.677-0.682 against 0.614-0.638)
constexpr bool FMT_NT_DEFAULT = false;

// Block boundaries: output offset o_b = o_first + b * OB clamped to [0, total]; its position
// j_b = o - o / 51; per boundary [decoded offset d_b of j_b, first N run and first lowercase run
// ending after j_b, j_b, and (fused path, tko given) the token-table entry holding d_b: the last
// with o_t <= d_b].  One thread per (boundary, run list).
__global__ void k_out_index(int64_t nres, int64_t total, int64_t o_first, int64_t nblk, int64_t ob, const int32_t* __restrict__ ns,
                            const int32_t* __restrict__ nl, const int64_t* __restrict__ ncum, int64_t nn,
                            const int32_t* __restrict__ ls, const int32_t* __restrict__ ll, int64_t nlr,
                            const int64_t* __restrict__ tko, const int64_t* __restrict__ d_ntok, int64_t* __restrict__ tab) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < 2 * (nblk + 1); i += (int64_t)gridDim.x * blockDim.x) {
        const int64_t b = i >> 1;
        int64_t o = o_first + b * ob;
        o = o < 0 ? 0 : (o > total ? total : o);
        const int64_t J = o - o / 51;
        if (i & 1) {
            tab[TW * b + 2] = first_run_ending_after(ls, ll, nlr, J);
        } else {
            const int64_t r = first_run_ending_after(ns, nl, nn, J);
            const int64_t d = J - n_before_at(ns, nl, ncum, nn, r, J);
            tab[TW * b + 0] = d;
            tab[TW * b + 1] = r;
            tab[TW * b + 3] = J;
            if (tko) {
                int64_t lo = 0, hi = *d_ntok;   // entry 0 (o = 0) qualifies
                while (lo < hi) {
                    const int64_t m = (lo + hi + 1) >> 1;
                    if (tko[m] <= d) lo = m; else hi = m - 1;
                }
                tab[TW * b + 4] = lo;
            }
        }
    }
}

template <bool NT>
__device__ __forceinline__ void store16(uint8_t* p, uint64_t lo, uint64_t hi) {
    if (NT) {   // streaming store: the output is not read again by this kernel
        __builtin_nontemporal_store(lo, reinterpret_cast<uint64_t*>(p));
        __builtin_nontemporal_store(hi, reinterpret_cast<uint64_t*>(p) + 1);
    } else {
        *reinterpret_cast<uint4*>(p) = make_uint4((uint32_t)lo, (uint32_t)(lo >> 32), (uint32_t)hi, (uint32_t)(hi >> 32));
    }
}

// format_out16 with the position (j, col of oc = max(o0, 0)) and the first N / lowercase runs
// ending after j (rn, rl) given by the caller
template <typename V, bool NT = false>
__device__ __forceinline__ void format_out16_at(int64_t o0, int64_t total, const uint8_t* sdec, int64_t dbase, const V& N,
                                                int64_t cn, int64_t ntot, const V& L, int64_t cl, uint8_t* out, int64_t j,
                                                int col, int64_t rn, int64_t rl) {
    const int64_t oc = o0 < 0 ? 0 : o0;
    int64_t n_s = INT64_MAX, n_e = INT64_MAX, n_b = ntot, l_s = INT64_MAX, l_e = INT64_MAX;
    if (rn < cn) { n_s = N.st(rn); n_e = N.en(rn); n_b = N.nb(rn); }
    if (rl < cl) { l_s = L.st(rl); l_e = L.en(rl); }
    uint64_t lo = 0, hi = 0;
    const int k0 = (int)(oc - o0), k1 = total - o0 < OPT ? (int)(total - o0) : OPT;
    if (k0 == 0 && k1 == OPT) {
        // Fast path: the thread's 16 output bytes are at most one '\n' (at knl) and 15-16 sequence
        // bytes j .. jl-1.  Lowercase runs (any number) and at most one N run inside them become
        // byte masks: the sequence bytes are the decoded bytes from j's decoded offset, those after
        // an N run inside the group from an offset shifted back by the run's length, N inside the
        // run, tolower where lowercase -- SWAR on four words, then a byte shift for the '\n'.  (A
        // per-byte loop with run bookkeeping ran whenever any lane of a wave met a run boundary:
        // with soft-masked runs every ~650 bases, nearly every wave; 620-680 VALU per wave.)
        const int knl = 50 - col;   // col in [0, 50]: the line's '\n' is output byte knl (if < 16)
        const int nseq = knl < OPT ? OPT - 1 : OPT;
        const int64_t jl = j + nseq;
        // N runs meeting [j, jl): one at most for this path
        int na = OPT, nbnd = OPT, nin = 0;   // N bytes [na, nbnd) of the group (relative)
        int64_t r = rn;
        int64_t nbj;                          // N bases before j
        if (rn < cn && n_s < j) nbj = n_b + (j - n_s);
        else nbj = rn < cn ? n_b : ntot;
        while (r < cn && (r == rn ? n_s : N.st(r)) < jl) {
            const int64_t rs = r == rn ? n_s : N.st(r), re = r == rn ? n_e : N.en(r);
            na = (int)((rs > j ? rs : j) - j);
            nbnd = (int)((re < jl ? re : jl) - j);
            nin++;
            r++;
        }
        const int64_t at1 = j - nbj - dbase;             // decoded offset of byte 0 (bytes before the N run)
        const int64_t at2 = at1 - (nbnd - na);            // (bytes after it: byte p at at2 + p)
        const uint32_t nm = nin ? (((1u << nbnd) - 1u) & ~((1u << na) - 1u)) : 0u;
        const uint32_t after = nin ? (~((1u << nbnd) - 1u) & 0xffffu) : 0u;   // bytes from the shifted window
        const bool use1 = (~after & ~nm & 0xffffu) != 0, use2 = after != 0;
        if (nin <= 1 && (!use1 || at1 >= 0) && (!use2 || at2 >= 0)) {
            // lowercase byte mask (bit per byte)
            uint32_t lm = 0;
            for (int64_t q = rl; q < cl; q++) {
                const int64_t ls = q == rl ? l_s : L.st(q);
                if (ls >= jl) break;
                const int64_t le = q == rl ? l_e : L.en(q);
                const int s0 = (int)((ls > j ? ls : j) - j), e0 = (int)((le < jl ? le : jl) - j);
                if (e0 > s0) lm |= ((1u << e0) - 1u) & ~((1u << s0) - 1u);
            }
            uint32_t w1[4] = {0, 0, 0, 0}, w2[4] = {0, 0, 0, 0};
            auto load16 = [&](int64_t at, uint32_t (&w)[4]) {
                const uint4 v = load16u(reinterpret_cast<const uint8_t*>(sdec) + at);
                w[0] = v.x; w[1] = v.y; w[2] = v.z; w[3] = v.w;
            };
            if (use1) load16(at1, w1);
            if (use2) load16(at2, w2);
            uint32_t w[4];
#pragma unroll
            for (int qq = 0; qq < 4; qq++) {
                // bit masks -> byte masks for bytes 4qq .. 4qq+3
                const uint32_t nb4 = (nm >> (4 * qq)) & 0xfu, ab4 = (after >> (4 * qq)) & 0xfu, lb4 = (lm >> (4 * qq)) & 0xfu;
                const uint32_t nB = (nb4 * 0x00204081u & 0x01010101u) * 0xffu;   // bit i -> byte i = 0xff
                const uint32_t aB = (ab4 * 0x00204081u & 0x01010101u) * 0xffu;
                const uint32_t lB = (lb4 * 0x00204081u & 0x01010101u) * 0xffu;
                uint32_t x = (w1[qq] & ~aB) | (w2[qq] & aB);
                x = (x & ~nB) | (0x4E4E4E4Eu & nB);                               // 'N'
                const uint32_t ge_a = ((x | 0x80808080u) - 0x41414141u) & 0x80808080u;   // byte >= 'A' (7-bit)
                const uint32_t gt_z = ((x | 0x80808080u) - 0x5B5B5B5Bu) & 0x80808080u;   // byte >= 'Z' + 1
                const uint32_t up = ge_a & ~gt_z & ~x & lB;                       // tolower where lowercase
                w[qq] = x + (up >> 2);
            }
            uint64_t slo = (uint64_t)w[0] | ((uint64_t)w[1] << 32), shi = (uint64_t)w[2] | ((uint64_t)w[3] << 32);
            if (knl < OPT) {   // bytes from knl on move up by one; '\n' at knl
                const uint64_t ulo = slo << 8, uhi = (shi << 8) | (slo >> 56);
                const uint64_t mlo = knl >= 8 ? ~0ull : (knl ? (1ull << (8 * knl)) - 1ull : 0ull);
                const uint64_t mhi = knl <= 8 ? 0ull : (1ull << (8 * (knl - 8))) - 1ull;
                slo = (slo & mlo) | (ulo & ~mlo);
                shi = (shi & mhi) | (uhi & ~mhi);
                if (knl < 8) slo = (slo & ~(0xffull << (8 * knl))) | ((uint64_t)'\n' << (8 * knl));
                else shi = (shi & ~(0xffull << (8 * (knl - 8)))) | ((uint64_t)'\n' << (8 * (knl - 8)));
            }
            store16<NT>(out + o0, slo, shi);
            return;
        }
    }
    for (int k = k0; k < k1; k++) {
        uint32_t c;
        if (col == 50) {
            c = '\n';
            col = 0;
        } else {
            while (j >= n_e) {
                rn++;
                if (rn < cn) { n_s = N.st(rn); n_e = N.en(rn); n_b = N.nb(rn); }
                else { n_s = n_e = INT64_MAX; n_b = ntot; }
            }
            while (j >= l_e) {
                rl++;
                if (rl < cl) { l_s = L.st(rl); l_e = L.en(rl); }
                else l_s = l_e = INT64_MAX;
            }
            c = j >= n_s ? (uint32_t)'N' : (uint32_t)sdec[j - n_b - dbase];
            if (j >= l_s) c = c_tolower((uint8_t)c);
            j++;
            col++;
        }
        if (k < 8) lo |= (uint64_t)c << (8 * k);
        else hi |= (uint64_t)c << (8 * (k - 8));
    }
    if (k0 == 0 && k1 == OPT) {
        store16<NT>(out + o0, lo, hi);
    } else {
        for (int k = k0; k < k1; k++) out[o0 + k] = (uint8_t)((k < 8 ? lo >> (8 * k) : hi >> (8 * (k - 8))) & 0xff);
    }
}

template <typename V, bool NT = false>
__device__ __forceinline__ void format_out16(int64_t o0, int64_t total, int64_t nres, const uint8_t* sdec, int64_t dbase,
                                             const V& N, int64_t cn, int64_t ntot, const V& L, int64_t cl, uint8_t* out) {
    (void)nres;
    const int64_t oc = o0 < 0 ? 0 : o0;
    if (oc >= total || o0 + OPT <= 0) return;
    const int64_t j = oc - oc / 51;
    const int col = (int)(oc % 51);
    format_out16_at<V, NT>(o0, total, sdec, dbase, N, cn, ntot, L, cl, out, j, col, first_end_after(N, 0, cn, j),
                           first_end_after(L, 0, cl, j));
}

// first r in [0, c) with e[r] > j over an LDS run list: short lists (a tile holds a few runs) by a
// linear pass, long ones by bisection
__device__ __forceinline__ int32_t lds_first_end_after(const int32_t* e, int32_t c, int32_t j) {
    if (c <= 16) {
        int32_t r = 0;
        while (r < c && e[r] <= j) r++;
        return r;
    }
    int32_t a = 0, b = c;
    while (a < b) {
        const int32_t m = (a + b) >> 1;
        if (e[m] > j) b = m; else a = m + 1;
    }
    return a;
}

// runs of the global lists from index a on, as views starting at 0 (format_out16's fallback)
struct GlobalRunsAt {
    const int32_t* s;
    const int32_t* l;
    const int64_t* b;
    int64_t a;
    __device__ int64_t st(int64_t r) const { return s[a + r]; }
    __device__ int64_t en(int64_t r) const { return (int64_t)s[a + r] + l[a + r]; }
    __device__ int64_t nb(int64_t r) const { return b ? b[a + r] : 0; }
};

// U: 16-byte outputs per thread (a block owns U * OB output bytes: fewer, larger dependent load
// phases per byte); NT: streaming stores for the output.
template <int U, bool NT>
__global__ __launch_bounds__(256) void k_format_out(const uint8_t* __restrict__ dec, int64_t nres, int64_t total, int64_t o_first,
                                                    const int32_t* __restrict__ ns, const int32_t* __restrict__ nl,
                                                    const int64_t* __restrict__ ncum, int64_t nn,
                                                    const int32_t* __restrict__ ls, const int32_t* __restrict__ ll,
                                                    int64_t nlr, const int64_t* __restrict__ tab, uint8_t* __restrict__ out) {
    // the tile's decoded bytes from a 16-byte-aligned base, 16 bytes per thread and load, with
    // 16 bytes of slack for format_out16's unaligned 16-byte reads (dec holds >= 64 bytes of slack)
    __shared__ uint4 sdec4[(U * OB + 64) / 16];
    __shared__ int32_t s_ns[OFRUNS], s_ne[OFRUNS], s_ls[OFRUNS], s_le[OFRUNS];
    __shared__ int64_t s_nb[OFRUNS];
    __shared__ int64_t st[2 * TW];
    uint32_t* sdec_w = reinterpret_cast<uint32_t*>(sdec4);
    const int tid = threadIdx.x;
    const int64_t b = blockIdx.x;   // (a grid-stride loop over blocks: 0.35-0.43 ms instead of 0.27)
    if (tid < 2 * TW) st[tid] = tab[TW * b + tid];
    __syncthreads();
    const int64_t d0 = st[0], d1 = st[TW];
    const int64_t n_lo = st[1], n_hi = st[TW + 1] < nn ? st[TW + 1] + 1 : nn;
    const int64_t l_lo = st[2], l_hi = st[TW + 2] < nlr ? st[TW + 2] + 1 : nlr;
    const int64_t ntot = nn ? ncum[nn - 1] + nl[nn - 1] : 0;
    const bool lds_runs = n_hi - n_lo <= OFRUNS && l_hi - l_lo <= OFRUNS;
    const int64_t a0 = d0 & ~(int64_t)15;
    const int64_t n16 = (d1 - a0 + 16 + 15) >> 4;   // <= (U * OB + 46) / 16
    const uint4* dec4 = reinterpret_cast<const uint4*>(dec + a0);
#pragma unroll
    for (int u = 0; u < U; u++) {
        const int64_t i = tid + 256 * u;
        if (i < n16) sdec4[i] = dec4[i];
    }
    if (U * 256 + tid < n16) sdec4[U * 256 + tid] = dec4[U * 256 + tid];
    if (lds_runs) {
        for (int64_t r = n_lo + tid; r < n_hi; r += 256) {
            const int32_t x = ns[r];
            s_ns[r - n_lo] = x;
            s_ne[r - n_lo] = x + nl[r];
            s_nb[r - n_lo] = ncum[r];
        }
        for (int64_t r = l_lo + tid; r < l_hi; r += 256) {
            const int32_t x = ls[r];
            s_ls[r - l_lo] = x;
            s_le[r - l_lo] = x + ll[r];
        }
    }
    __syncthreads();
    const uint8_t* sdec = reinterpret_cast<const uint8_t*>(sdec_w);
    // the block's first output offset (clamped) and its (j, col): a thread's (j, col) follow in 32-bit
    // arithmetic from its offset inside the block (no 64-bit division per thread)
    const int64_t ob = o_first + b * (U * OB), obc = ob < 0 ? 0 : ob;
    const int64_t Jb = st[3];   // obc - obc / 51 (k_out_index)
    const int32_t colb = (int32_t)(obc - 51 * (obc - Jb));
#pragma unroll
    for (int u = 0; u < U; u++) {
        const int64_t o0 = ob + (int64_t)(u * 256 + tid) * OPT;
        if (lds_runs) {
            const int64_t oc = o0 < 0 ? 0 : o0;
            if (oc >= total || o0 + OPT <= 0) continue;
            const int32_t q = colb + (int32_t)(oc - obc);
            const int32_t nl51 = q / 51;
            const int64_t j = Jb + (oc - obc) - nl51;
            const int col = q - 51 * nl51;
            const int32_t jr = (int32_t)j;   // (positions are int32 in the run lists)
            const LdsRuns N{s_ns, s_ne, s_nb}, L{s_ls, s_le, nullptr};
            format_out16_at<LdsRuns, NT>(o0, total, sdec, a0, N, n_hi - n_lo, ntot, L, l_hi - l_lo, out, j, col,
                                         lds_first_end_after(s_ne, (int32_t)(n_hi - n_lo), jr),
                                         lds_first_end_after(s_le, (int32_t)(l_hi - l_lo), jr));
        } else {
            const GlobalRunsAt N{ns, nl, ncum, n_lo}, L{ls, ll, nullptr, l_lo};
            format_out16<GlobalRunsAt, NT>(o0, total, nres, sdec, a0, N, n_hi - n_lo, ntot, L, l_hi - l_lo, out);
        }
    }
}

// ---------------------------------------------------------------------------------------------
// Pipelined formatter (opt-in, SCCG_FMT_PIPE=1): a resident grid (8 blocks per CU) walks the output tiles of
// k_format_out, block b taking tiles b, b + G, b + 2G, ...; while it formats one tile from LDS the
// loads of the next (its decoded words and runs, into registers) and the k_out_index row of the one
// after are in flight, so a tile costs max(format, memory) instead of two dependent HBM round trips
// plus the format (k_format_out: 62 k blocks in ~30 generations, ~9 us each for chr1).  Two LDS
// buffers alternate; tiles touching more than PRUNS runs of a kind read that run list from global.
// ---------------------------------------------------------------------------------------------
constexpr int PRUNS = 128;

struct PipeRegs {
    uint32_t w[5];
    int32_t ns, ne, ls, le;
    int64_t nb;
};

struct PipeTile {
    int64_t d0, d1, a0, nw, n_lo, n_hi, l_lo, l_hi;
    bool lds;
    __device__ PipeTile(const int64_t* r, int64_t nn, int64_t nlr) {
        d0 = r[0];
        d1 = r[TW];
        a0 = d0 & ~(int64_t)3;
        nw = (d1 - a0 + 3) >> 2;
        n_lo = r[1];
        n_hi = r[TW + 1] < nn ? r[TW + 1] + 1 : nn;
        l_lo = r[2];
        l_hi = r[TW + 2] < nlr ? r[TW + 2] + 1 : nlr;
        lds = n_hi - n_lo <= PRUNS && l_hi - l_lo <= PRUNS;
    }
};

__device__ __forceinline__ void pipe_load(const PipeTile& T, const uint8_t* __restrict__ dec, const int32_t* __restrict__ ns,
                                          const int32_t* __restrict__ nl, const int64_t* __restrict__ ncum,
                                          const int32_t* __restrict__ ls, const int32_t* __restrict__ ll, int tid, PipeRegs& R) {
    const uint32_t* decw = reinterpret_cast<const uint32_t*>(dec + T.a0);
#pragma unroll
    for (int q = 0; q < 5; q++) R.w[q] = tid + 256 * q < T.nw ? decw[tid + 256 * q] : 0u;
    if (T.lds) {
        const int64_t rn = T.n_lo + tid, rl = T.l_lo + tid;
        if (rn < T.n_hi) { R.ns = ns[rn]; R.ne = R.ns + nl[rn]; R.nb = ncum[rn]; }
        if (rl < T.l_hi) { R.ls = ls[rl]; R.le = R.ls + ll[rl]; }
    }
}

__device__ __forceinline__ void pipe_store(const PipeTile& T, const PipeRegs& R, int tid, uint32_t* sdec, int32_t* sns,
                                           int32_t* sne, int64_t* snb, int32_t* sls, int32_t* sle) {
#pragma unroll
    for (int q = 0; q < 5; q++)
        if (tid + 256 * q < T.nw) sdec[tid + 256 * q] = R.w[q];
    if (T.lds) {
        if (T.n_lo + tid < T.n_hi) { sns[tid] = R.ns; sne[tid] = R.ne; snb[tid] = R.nb; }
        if (T.l_lo + tid < T.l_hi) { sls[tid] = R.ls; sle[tid] = R.le; }
    }
}

__global__ __launch_bounds__(256) void k_format_pipe(const uint8_t* __restrict__ dec, int64_t nres, int64_t total, int64_t o_first,
                                                     int64_t nblk, const int32_t* __restrict__ ns, const int32_t* __restrict__ nl,
                                                     const int64_t* __restrict__ ncum, int64_t nn,
                                                     const int32_t* __restrict__ ls, const int32_t* __restrict__ ll,
                                                     int64_t nlr, const int64_t* __restrict__ tab, uint8_t* __restrict__ out) {
    static_assert(5 * 256 >= OB / 4 + 2, "five words per thread cover a tile's decoded bytes");
    __shared__ uint32_t sdec[2][OB / 4 + 4];
    __shared__ int32_t s_ns[2][PRUNS], s_ne[2][PRUNS], s_ls[2][PRUNS], s_le[2][PRUNS];
    __shared__ int64_t s_nb[2][PRUNS];
    __shared__ int64_t st[3][2 * TW];
    const int tid = threadIdx.x;
    const int64_t G = gridDim.x, b0 = blockIdx.x;
    if (b0 >= nblk) return;
    const int64_t ntot = nn ? ncum[nn - 1] + nl[nn - 1] : 0;
    if (tid < 2 * TW) {
        st[0][tid] = tab[TW * b0 + tid];
        if (b0 + G < nblk) st[1][tid] = tab[TW * (b0 + G) + tid];
    }
    __syncthreads();
    PipeRegs R{};
    {
        const PipeTile T(st[0], nn, nlr);
        pipe_load(T, dec, ns, nl, ncum, ls, ll, tid, R);
        pipe_store(T, R, tid, sdec[0], s_ns[0], s_ne[0], s_nb[0], s_ls[0], s_le[0]);
    }
    __syncthreads();
    for (int64_t i = 0;; i++) {
        const int64_t bc = b0 + i * G;
        if (bc >= nblk) break;
        const int cur = (int)(i & 1), nxt = cur ^ 1;
        const bool has_next = bc + G < nblk;
        // the next tile's loads and the row after it, in flight while this tile is formatted
        int64_t tv = 0;
        if (has_next) {
            const PipeTile Tn(st[(i + 1) % 3], nn, nlr);   // (rebuilt from LDS after the format: fewer live registers)
            pipe_load(Tn, dec, ns, nl, ncum, ls, ll, tid, R);
            if (tid < 2 * TW && bc + 2 * G < nblk) tv = tab[TW * (bc + 2 * G) + tid];
        }
        {
            const PipeTile T(st[i % 3], nn, nlr);
            const uint8_t* sd = reinterpret_cast<const uint8_t*>(sdec[cur]);
            const int64_t o0 = o_first + bc * OB + (int64_t)tid * OPT;
            if (T.lds) {
                const LdsRuns N{s_ns[cur], s_ne[cur], s_nb[cur]}, L{s_ls[cur], s_le[cur], nullptr};
                format_out16(o0, total, nres, sd, T.a0, N, T.n_hi - T.n_lo, ntot, L, T.l_hi - T.l_lo, out);
            } else {
                const GlobalRunsAt N{ns, nl, ncum, T.n_lo}, L{ls, ll, nullptr, T.l_lo};
                format_out16(o0, total, nres, sd, T.a0, N, T.n_hi - T.n_lo, ntot, L, T.l_hi - T.l_lo, out);
            }
        }
        if (!has_next) break;
        __syncthreads();   // buffer nxt (tile i - 1's) and row (i + 2) % 3 (= (i - 1) % 3) are free
        {
            const PipeTile Tn(st[(i + 1) % 3], nn, nlr);
            pipe_store(Tn, R, tid, sdec[nxt], s_ns[nxt], s_ne[nxt], s_nb[nxt], s_ls[nxt], s_le[nxt]);
        }
        if (tid < 2 * TW) st[(i + 2) % 3][tid] = tv;
        __syncthreads();
    }
}

// ---------------------------------------------------------------------------------------------
// Fused reconstruction formatter (opt-in, SCCG_DC_FUSED=1): k_format_out with the block's decoded bytes expanded
// from the token table instead of read from a decoded buffer -- the tokens the block touches
// (k_out_index entries t_b .. t_b+1) are staged in LDS beside its runs, then each thread gathers 16
// decoded bytes (a token's R' bytes with five dword loads, else bytes from R' / the record's
// literals) into the block's LDS copy, and formats as k_format_out.  The decoded buffer is never
// written or re-read (the fill wrote ~|T| bytes and the formatter read them back), and the token
// table is built beside the reference strip, so the strip is followed directly by this kernel.
// ---------------------------------------------------------------------------------------------
constexpr int OTOK = 128;

struct TokLds {
    const int64_t *o, *p, *l, *r;
    int64_t base;
    __device__ int64_t O(int64_t t) const { return o[t - base]; }
    __device__ int64_t P(int64_t t) const { return p[t - base]; }
    __device__ int64_t L(int64_t t) const { return l[t - base]; }
    __device__ int64_t R(int64_t t) const { return r[t - base]; }
};
struct TokGlobal {
    const int64_t *o, *p, *l, *r;
    __device__ int64_t O(int64_t t) const { return o[t]; }
    __device__ int64_t P(int64_t t) const { return p[t]; }
    __device__ int64_t L(int64_t t) const { return l[t]; }
    __device__ int64_t R(int64_t t) const { return r[t]; }
};

// decoded bytes [x, x + 16) into w[0..3] (bytes outside [d0, d1) are 0: no format position reads them)
template <typename TV>
__device__ __forceinline__ void expand16(int64_t x, int64_t d0, int64_t d1, int64_t t_lo, int64_t t_hi, const TV& T,
                                         const uint8_t* __restrict__ R, int64_t nref, const uint8_t* __restrict__ rec,
                                         int64_t nrec, uint32_t* w) {
    const int64_t xs = x < d0 ? d0 : x;
    int64_t lo = t_lo, hi = t_hi;   // last entry with o <= xs (o of t_lo <= d0 by construction)
    while (lo < hi) {
        const int64_t m = (lo + hi + 1) >> 1;
        if (T.O(m) <= xs) lo = m; else hi = m - 1;
    }
    int64_t t = lo, o = T.O(t), l = T.L(t), p = T.P(t), r = T.R(t);
    int64_t onext = t < t_hi ? T.O(t + 1) : INT64_MAX;
    bool pv = p >= 0 && p + l <= nref;
    if (x >= o && x + 16 <= o + l && pv) {   // all 16 from one token: dword loads (R' has >= 64 B of slack)
        const uint8_t* s0 = R + p + (x - o);
        const unsigned sh = (unsigned)((uintptr_t)s0 & 3);
        const uint32_t* a = reinterpret_cast<const uint32_t*>((uintptr_t)s0 & ~(uintptr_t)3);
        const uint32_t w0 = a[0], w1 = a[1], w2 = a[2], w3 = a[3], w4 = a[4];
        w[0] = __builtin_amdgcn_alignbyte(w1, w0, sh);
        w[1] = __builtin_amdgcn_alignbyte(w2, w1, sh);
        w[2] = __builtin_amdgcn_alignbyte(w3, w2, sh);
        w[3] = __builtin_amdgcn_alignbyte(w4, w3, sh);
        return;
    }
    // every source first (a 32-bit code: R' offset, or the record offset | 1 << 31; ~0 = none; the
    // host takes this path only when |R'| and the record line are below 2^31), then all 16 loads
    uint32_t src[16];
#pragma unroll
    for (int k = 0; k < 16; k++) {
        const int64_t y = x + k;
        src[k] = ~0u;
        if (y >= xs && y < d1) {
            while (y >= onext) {
                t++;
                o = onext; l = T.L(t); p = T.P(t); r = T.R(t);
                onext = t < t_hi ? T.O(t + 1) : INT64_MAX;
                pv = p >= 0 && p + l <= nref;
            }
            if (y < o + l) {
                if (pv) src[k] = (uint32_t)(p + (y - o));
            } else {
                const int64_t q = r + (y - o - l);
                if (q >= 0 && q < nrec) src[k] = (uint32_t)q | 0x80000000u;
            }
        }
    }
    uint32_t v[4] = {0, 0, 0, 0};
#pragma unroll
    for (int k = 0; k < 16; k++) {
        const uint32_t c = src[k];
        const uint32_t b = c == ~0u ? 0u : (c >> 31) ? rec[c & 0x7fffffffu] : R[c];
        v[k >> 2] |= b << (8 * (k & 3));
    }
    w[0] = v[0]; w[1] = v[1]; w[2] = v[2]; w[3] = v[3];
}

#ifndef SCCG_FUSED_WAVES
#define SCCG_FUSED_WAVES 1
#endif
__global__ __launch_bounds__(256, SCCG_FUSED_WAVES) void k_format_fused(DcFmtSrc F, int64_t nres, int64_t total, int64_t o_first,
                                                      const int32_t* __restrict__ ns, const int32_t* __restrict__ nl,
                                                      const int64_t* __restrict__ ncum, int64_t nn,
                                                      const int32_t* __restrict__ ls, const int32_t* __restrict__ ll,
                                                      int64_t nlr, const int64_t* __restrict__ tab, uint8_t* __restrict__ out) {
    __shared__ uint32_t sdec_w[OB / 4 + 8];
    __shared__ int32_t s_ns[OFRUNS], s_ne[OFRUNS], s_ls[OFRUNS], s_le[OFRUNS];
    __shared__ int64_t s_nb[OFRUNS];
    __shared__ int64_t s_to[OTOK], s_tp[OTOK], s_tl[OTOK], s_tr[OTOK];
    __shared__ int64_t st[2 * TW + 1];
    const int tid = threadIdx.x;
    const int64_t b = blockIdx.x;
    if (tid < 2 * TW) st[tid] = tab[TW * b + tid];
    if (tid == 2 * TW) st[2 * TW] = *F.d_nref;
    __syncthreads();
    const int64_t d0 = st[0], d1 = st[TW];
    const int64_t n_lo = st[1], n_hi = st[TW + 1] < nn ? st[TW + 1] + 1 : nn;
    const int64_t l_lo = st[2], l_hi = st[TW + 2] < nlr ? st[TW + 2] + 1 : nlr;
    const int64_t t_lo = st[4], t_hi = st[TW + 4];
    const int64_t nref = st[2 * TW];
    const int64_t ntot = nn ? ncum[nn - 1] + nl[nn - 1] : 0;
    const bool lds_runs = n_hi - n_lo <= OFRUNS && l_hi - l_lo <= OFRUNS;
    const bool lds_tok = t_hi - t_lo < OTOK;
    if (lds_tok) {
        for (int64_t t = t_lo + tid; t <= t_hi; t += 256) {
            s_to[t - t_lo] = F.tk.o[t];
            s_tp[t - t_lo] = F.tk.p[t];
            s_tl[t - t_lo] = F.tk.l[t];
            s_tr[t - t_lo] = F.tk.r[t];
        }
    }
    if (lds_runs) {
        for (int64_t r = n_lo + tid; r < n_hi; r += 256) {
            const int32_t x = ns[r];
            s_ns[r - n_lo] = x;
            s_ne[r - n_lo] = x + nl[r];
            s_nb[r - n_lo] = ncum[r];
        }
        for (int64_t r = l_lo + tid; r < l_hi; r += 256) {
            const int32_t x = ls[r];
            s_ls[r - l_lo] = x;
            s_le[r - l_lo] = x + ll[r];
        }
    }
    __syncthreads();
    const int64_t a0 = d0 & ~(int64_t)3;
    const int64_t nch = (d1 - a0 + 15) >> 4;
    for (int64_t c = tid; c < nch; c += 256) {
        uint32_t* w = sdec_w + 4 * c;
        if (lds_tok) expand16(a0 + 16 * c, d0, d1, t_lo, t_hi, TokLds{s_to, s_tp, s_tl, s_tr, t_lo}, F.R, nref, F.rec, F.nrec, w);
        else expand16(a0 + 16 * c, d0, d1, t_lo, t_hi, TokGlobal{F.tk.o, F.tk.p, F.tk.l, F.tk.r}, F.R, nref, F.rec, F.nrec, w);
    }
    __syncthreads();
    const uint8_t* sdec = reinterpret_cast<const uint8_t*>(sdec_w);
    const int64_t o0 = o_first + b * OB + (int64_t)tid * OPT;
    if (lds_runs) {
        const LdsRuns N{s_ns, s_ne, s_nb}, L{s_ls, s_le, nullptr};
        format_out16(o0, total, nres, sdec, a0, N, n_hi - n_lo, ntot, L, l_hi - l_lo, out);
    } else {
        const GlobalRunsAt N{ns, nl, ncum, n_lo}, L{ls, ll, nullptr, l_lo};
        format_out16(o0, total, nres, sdec, a0, N, n_hi - n_lo, ntot, L, l_hi - l_lo, out);
    }
}

}  // namespace

// =============================================================================================
int dc_find_lines(const uint8_t* d_rec, int64_t n, int64_t* d_nl /*8: 4 results + 4 tickets*/, hipStream_t s) {
    for (int i = 0; i < 4; i++) {
        int rc = launch_first_match(d_rec, n, i ? (const int64_t*)(d_nl + i - 1) : nullptr, 1, '\n', d_nl + i, d_nl + 4 + i, s);
        if (rc) return rc;
    }
    return 0;
}

namespace {
__global__ void k_nl_init(int64_t* cnt, int32_t* err) {
    if (threadIdx.x == 0) {
        *cnt = 0;
        if (err) *err = 0;
    }
}
}  // namespace

int dc_newlines(const uint8_t* d_rec, int64_t n, int64_t* d_buf, hipStream_t s, int32_t* d_err) {
    hipLaunchKernelGGL(k_nl_init, dim3(1), dim3(64), 0, s, d_buf, d_err);   // (one launch zeroes both)
    SCCG_HIP(hipGetLastError());
    if (n <= 0) return 0;
    const unsigned g = grid_for(n, 256) > 4096 ? 4096 : grid_for(n, 256);
    hipLaunchKernelGGL(k_newlines, dim3(g), dim3(256), 0, s, d_rec, n, reinterpret_cast<unsigned long long*>(d_buf), d_buf + 1);
    SCCG_HIP(hipGetLastError());
    return 0;
}

int dc_last_paren(const uint8_t* d_s, int64_t n, int64_t* d_lp, int64_t* d_partial, hipStream_t s) {
    if (n <= 0) return 0;
    const unsigned g = grid_for(n, 256) > 8192 ? 8192 : grid_for(n, 256);
    hipLaunchKernelGGL(k_paren_pos, dim3(g), dim3(256), 0, s, d_s, n, d_lp);
    SCCG_HIP(hipGetLastError());
    // exclusive max-scan: last parenthesis strictly before i; the inclusive form is not needed
    return dev_excl_max(d_lp, d_lp, n, nullptr, d_partial, s);
}

int64_t dc_run_cap(int64_t n) { return n / 2 + 2; }

namespace {
bool rl_tiled() {   // (SCCG_RL_SCAN=1, A/B runs: the scan-based parser)
    static const bool v = getenv("SCCG_RL_SCAN") == nullptr;
    return v;
}
bool rl_tiled_ok(int64_t n) { return rl_tiled() && (n + RL_TILE - 1) / RL_TILE <= 64 * 1024; }

// the scan-based parser of one line (lines over 64 MiB, or SCCG_RL_SCAN)
int parse_runs_scan(const uint8_t* d_s, int64_t n, DcRuns* r, int64_t* d_lp, int64_t* d_flag, int64_t* d_dlt,
                    int64_t* d_partial, int32_t* d_err, int64_t* d_count, hipStream_t s) {
    if (n <= 0) {
        SCCG_HIP(hipMemsetAsync(d_count, 0, 2 * sizeof(int64_t), s));
        return 0;
    }
    const int64_t cap = dc_run_cap(n);
    int rc = dc_last_paren(d_s, n, d_lp, d_partial, s);
    if (rc) return rc;
    SCCG_HIP(hipMemsetAsync(d_dlt, 0, (size_t)cap * sizeof(int64_t), s));   // deltas past the runs scan as 0
    const unsigned g = grid_for(n, 256) > 8192 ? 8192 : grid_for(n, 256);
    hipLaunchKernelGGL(k_run_items_flag, dim3(g), dim3(256), 0, s, d_s, n, (const int64_t*)d_lp, d_flag, d_err);
    rc = dev_excl_sum(d_flag, d_flag, n, d_count, d_partial, s);   // item ranks; d_count[0] = runs
    if (rc) return rc;
    hipLaunchKernelGGL(k_run_items_parse, dim3(g), dim3(256), 0, s, d_s, n, (const int64_t*)d_lp,
                       (const int64_t*)d_flag, d_dlt, r->len, d_err);
    SCCG_HIP(hipGetLastError());
    // exclusive sum of deltas into d_flag (free now), then starts and int64 lengths, then the
    // N-count prefix; d_count[1] = total run length
    rc = dev_excl_sum(d_dlt, d_flag, cap, nullptr, d_partial, s);
    if (rc) return rc;
    const unsigned g2 = grid_for(cap, 256) > 8192 ? 8192 : grid_for(cap, 256);
    hipLaunchKernelGGL(k_run_finish, dim3(g2), dim3(256), 0, s, (const int64_t*)d_flag, (const int64_t*)d_dlt,
                       (const int32_t*)r->len, cap, (const int64_t*)d_count, r->start, r->cum, d_err);
    SCCG_HIP(hipGetLastError());
    return dev_excl_sum(r->cum, r->cum, cap, d_count + 1, d_partial, s);
}

RlJob rl_job_of(const uint8_t* d_s, int64_t n, DcRuns* r, int64_t* tsum, int64_t* d_count) {
    return RlJob{d_s, n > 0 ? n : 0, n > 0 ? (n + RL_TILE - 1) / RL_TILE : 0, tsum, r->start, r->len, r->cum, d_count};
}

int parse_runs_tiled(const RlJob& j0, const RlJob& j1, int32_t* d_err, hipStream_t s) {
    const int64_t nt = j0.ntiles + j1.ntiles;
    if (nt > 0) {
        const unsigned g = (unsigned)((nt + 3) / 4);
        hipLaunchKernelGGL(k_rl_tiles, dim3(g), dim3(256), 0, s, j0, j1, d_err);
        hipLaunchKernelGGL(k_rl_scan, dim3(2), dim3(RL_SCAN_T), 0, s, j0, j1);
        hipLaunchKernelGGL(k_rl_write, dim3(g), dim3(256), 0, s, j0, j1, d_err);
    } else {
        hipLaunchKernelGGL(k_rl_scan, dim3(2), dim3(RL_SCAN_T), 0, s, j0, j1);   // (zero counts)
    }
    SCCG_HIP(hipGetLastError());
    return 0;
}
}  // namespace

int dc_parse_runs(const uint8_t* d_s, int64_t n, DcRuns* r, int64_t* d_lp, int64_t* d_flag, int64_t* d_dlt,
                  int64_t* d_partial, int32_t* d_err, int64_t* d_count, hipStream_t s) {
    if (n > 0 && rl_tiled_ok(n)) {   // tiled: d_flag holds the per-tile summaries (4 per tile)
        DcRuns none{};
        return parse_runs_tiled(rl_job_of(d_s, n, r, d_flag, d_count), rl_job_of(nullptr, 0, &none, nullptr, nullptr), d_err, s);
    }
    return parse_runs_scan(d_s, n, r, d_lp, d_flag, d_dlt, d_partial, d_err, d_count, s);
}

int dc_parse_runs2(const uint8_t* s0, int64_t n0, DcRuns* r0, int64_t* d_count0, const uint8_t* s1, int64_t n1, DcRuns* r1,
                   int64_t* d_count1, int64_t* d_lp, int64_t* d_flag, int64_t* d_dlt, int64_t* d_partial, int32_t* d_err,
                   hipStream_t s) {
    if (rl_tiled_ok(n0) && rl_tiled_ok(n1))   // both lines in one launch set; summaries in d_flag / d_dlt
        return parse_runs_tiled(rl_job_of(s0, n0, r0, d_flag, d_count0), rl_job_of(s1, n1, r1, d_dlt, d_count1), d_err, s);
    int rc = dc_parse_runs(s0, n0, r0, d_lp, d_flag, d_dlt, d_partial, d_err, d_count0, s);
    if (!rc) rc = dc_parse_runs(s1, n1, r1, d_lp, d_flag, d_dlt, d_partial, d_err, d_count1, s);
    return rc;
}

int dc_n_check(const DcRuns& nr, const int64_t* d_ncnt, const int64_t* d_D, int32_t* d_err, hipStream_t s) {
    hipLaunchKernelGGL(k_n_check, dim3(1), dim3(64), 0, s, (const int32_t*)nr.start, (const int32_t*)nr.len, d_ncnt, d_D,
                       d_err);
    SCCG_HIP(hipGetLastError());
    return 0;
}

int dc_decode_prepare(const uint8_t* d_s, int64_t n, int64_t* d_lp, int64_t* d_contrib, int64_t* d_dlt, int64_t* d_off,
                      int64_t* d_dsum, const int64_t* d_nref, hipEvent_t nref_ready, int64_t* d_partial, int32_t* d_err,
                      int64_t* d_total, hipStream_t s, const DcTokBuf* tk) {
    if (n <= 0) {
        SCCG_HIP(hipMemsetAsync(d_total, 0, sizeof(int64_t), s));
        if (tk) {   // no tokens: the sentinel entry alone
            SCCG_HIP(hipMemsetAsync(tk->d_ntok, 0, sizeof(int64_t), s));
            for (int64_t* a : {tk->tab.o, tk->tab.p, tk->tab.l, tk->tab.r}) SCCG_HIP(hipMemsetAsync(a, 0, sizeof(int64_t), s));
        }
        return 0;
    }
    if (dc_tok_tiled()) {
        // per 64-byte block: state, output bytes, deltas; their exclusive prefixes -> d_off, d_dsum
        const int64_t nb = (n + TK_B - 1) / TK_B;
        const unsigned g = (unsigned)((n + 4 * 1024 - 1) / (4 * 1024));   // 4 waves of 1 KiB per block
        hipLaunchKernelGGL(k_tok_blocks, dim3(g), dim3(256), 0, s, d_s, n, d_lp, d_contrib, d_dlt, d_err,
                           tk ? tk->btok : nullptr);
        SCCG_HIP(hipGetLastError());
        // (d_partial: scan_partials_needed(n + 1) + 16 >= 2 * scan_partials_needed(nb))
        int rc = dev_excl_sum2(d_contrib, d_off, d_total, d_dlt, d_dsum, nullptr, nb, d_partial, s);
        if (rc || !tk) return rc;   // (unfused: the range check is in the fill, dc_decode_fill)
        rc = dev_excl_sum(tk->btok, tk->btoff, nb, tk->d_ntok, d_partial, s);
        if (rc) return rc;
        PROF_LAUNCH(PROF_DC_DECODE, s, k_tok_emit, dim3(grid_for(nb, WPB)), dim3(SCCG_BLOCK), 0, s, d_s, n, (const int64_t*)d_lp,
                    (const int64_t*)d_off, (const int64_t*)d_dsum, (const int64_t*)tk->btoff, tk->tab);
        SCCG_HIP(hipGetLastError());
        (void)d_nref;
        (void)nref_ready;
        return 0;   // (the range check: dc_tok_range, after the reference strip)
    }
    int rc = dc_last_paren(d_s, n, d_lp, d_partial, s);
    if (rc) return rc;
    const unsigned g = grid_for(n, 256) > 8192 ? 8192 : grid_for(n, 256);
    hipLaunchKernelGGL(k_tok_parse, dim3(g), dim3(256), 0, s, d_s, n, (const int64_t*)d_lp, d_contrib, d_dlt, d_err);
    SCCG_HIP(hipGetLastError());
    rc = dev_excl_sum(d_contrib, d_off, n, d_total, d_partial, s);
    if (rc) return rc;
    rc = dev_excl_sum(d_dlt, d_dsum, n, nullptr, d_partial, s);
    if (rc) return rc;
    if (nref_ready) SCCG_HIP(hipStreamWaitEvent(s, nref_ready, 0));
    hipLaunchKernelGGL(k_tok_check, dim3(g), dim3(256), 0, s, d_s, n, (const int64_t*)d_dsum, (const int64_t*)d_dlt,
                       (const int64_t*)d_contrib, d_nref, d_err);
    SCCG_HIP(hipGetLastError());
    return 0;
}

int64_t dc_tok_cap(int64_t n) { return n / 5 + 2; }   // a token "(d,l)" takes >= 5 bytes; tokens are disjoint

bool dc_fused() {   // (opt-in, SCCG_DC_FUSED=1: measured slower so far)
    static const bool v = dc_tok_tiled() && getenv("SCCG_DC_FUSED") != nullptr;
    return v;
}

int dc_tok_range(const DcTokBuf& tk, int64_t cap, const int64_t* d_nref, int32_t* d_err, hipStream_t s) {
    const unsigned g = grid_for(cap, 256) > 1024 ? 1024 : grid_for(cap, 256);
    hipLaunchKernelGGL(k_tok_range, dim3(g), dim3(256), 0, s, tk.tab, (const int64_t*)tk.d_ntok, d_nref, d_err);
    SCCG_HIP(hipGetLastError());
    return 0;
}

bool dc_tok_tiled() {
    // (SCCG_TOK_SCAN=1, A/B runs: the scan-based record-line path; chr1 1.04-1.05 ms vs 1.02-1.03 tiled)
    static const bool v = getenv("SCCG_TOK_SCAN") == nullptr;
    return v;
}

int dc_decode_fill(const uint8_t* d_s, int64_t n, const int64_t* d_lp, const int64_t* d_off, const int64_t* d_dsum,
                   const int64_t* d_dlt, const int64_t* d_contrib, const uint8_t* d_R, uint8_t* d_dec, hipStream_t s,
                   const int64_t* d_nref, int32_t* d_err, int64_t dcap) {
    if (n <= 0) return 0;
    if (dc_tok_tiled()) {
        PROF_LAUNCH(PROF_DC_DECODE, s, k_tok_fill2<true>, dim3(grid_for((n + TK_B - 1) / TK_B, WPB)), dim3(SCCG_BLOCK), 0, s, d_s, n,
                    d_lp, d_off, d_dsum, d_nref, d_R, d_dec, d_err, dcap);
        SCCG_HIP(hipGetLastError());
        return 0;
    }
    PROF_LAUNCH(PROF_DC_DECODE, s, k_tok_fill, dim3(grid_for(n, 64 * WPB)), dim3(SCCG_BLOCK), 0, s, d_s, n, d_lp, d_off, d_dsum, d_dlt,
                       d_contrib, d_R, d_dec);
    SCCG_HIP(hipGetLastError());
    return 0;
}

int dc_tok_range_tiled(const uint8_t* d_s, int64_t n, const int64_t* d_lp, const int64_t* d_off, const int64_t* d_dsum,
                       const int64_t* d_nref, int32_t* d_err, hipStream_t s) {
    if (n <= 0 || !dc_tok_tiled()) return 0;   // (the scan path checked the range in dc_decode_prepare)
    hipLaunchKernelGGL(k_tok_fill2<false>, dim3(grid_for((n + TK_B - 1) / TK_B, WPB)), dim3(SCCG_BLOCK), 0, s, d_s, n, d_lp,
                       d_off, d_dsum, d_nref, (const uint8_t*)nullptr, (uint8_t*)nullptr, d_err, (int64_t)0);
    SCCG_HIP(hipGetLastError());
    return 0;
}

int64_t dc_format_span_words(int64_t nres) {   // (both formatters' tables; the output's misalignment adds a block)
    const int64_t a = 3 * ((nres + FSPAN - 1) / FSPAN + 2), o = TW * ((nres + nres / 50 + 16) / OB + 3);
    return a > o ? a : o;
}

namespace {
bool fmt_span_path() {   // (A/B runs: the position-centric writer)
    static const bool v = getenv("SCCG_FMT_SPAN") != nullptr;
    return v;
}
bool fmt_pipe() {   // (SCCG_FMT_PIPE=1, A/B runs: the resident pipelined grid)
    static const bool v = getenv("SCCG_FMT_PIPE") != nullptr;
    return v;
}
int fmt_u() {   // output bytes per k_format_out block: U * OB (the fused and pipelined formatters use OB)
    static const int v = [] {
        const char* e = getenv("SCCG_FMT_U");
        const int u = e ? atoi(e) : FMT_U_DEFAULT;
        return u == 1 || u == 2 || u == 4 ? u : FMT_U_DEFAULT;
    }();
    return v;
}
struct FmtGeom {
    int64_t total, o_first, ob, nblk;
};
FmtGeom fmt_geom(int64_t nres, const uint8_t* d_out, bool ob1) {
    FmtGeom g;
    g.total = nres + (nres - 1) / 50;   // the final '\n' is the caller's
    g.o_first = -(int64_t)((uintptr_t)d_out & 15);
    g.ob = ob1 ? OB : (int64_t)fmt_u() * OB;
    g.nblk = (g.total - g.o_first + g.ob - 1) / g.ob;
    return g;
}
int launch_out_index(const FmtGeom& g, int64_t nres, const DcRuns& nr, const DcRuns& lr, const DcFmtSrc* fz,
                     int64_t* d_span, hipStream_t s) {
    hipLaunchKernelGGL(k_out_index, dim3(grid_for(2 * (g.nblk + 1), 256)), dim3(256), 0, s, nres, g.total, g.o_first, g.nblk,
                       g.ob, (const int32_t*)nr.start, (const int32_t*)nr.len, (const int64_t*)nr.cum, nr.n,
                       (const int32_t*)lr.start, (const int32_t*)lr.len, lr.n, fz ? (const int64_t*)fz->tk.o : nullptr,
                       fz ? fz->d_ntok : nullptr, d_span);
    SCCG_HIP(hipGetLastError());
    return 0;
}
}  // namespace

bool dc_format_index(int64_t nres, const DcRuns& nr, const DcRuns& lr, int64_t* d_span, uint8_t* d_out, hipStream_t s,
                     int* rc) {
    *rc = 0;
    if (nres <= 0 || fmt_span_path() || fmt_pipe()) return false;
    *rc = launch_out_index(fmt_geom(nres, d_out, false), nres, nr, lr, nullptr, d_span, s);
    return true;
}

int dc_format(const uint8_t* d_dec, int64_t nres, const DcRuns& nr, const DcRuns& lr, int64_t* d_span, uint8_t* d_out,
              hipStream_t s, const DcFmtSrc* fz, hipEvent_t wait_before, bool index_ready) {
    if (nres <= 0) {
        if (wait_before) SCCG_HIP(hipStreamWaitEvent(s, wait_before, 0));
        return 0;
    }
    const bool span_path = fmt_span_path();
    if (fz || !span_path) {
        static const bool fmt_nt = [] {
            const char* e = getenv("SCCG_FMT_NT");
            return e ? atoi(e) != 0 : FMT_NT_DEFAULT;
        }();
        const bool pipe = fmt_pipe();
        const FmtGeom g = fmt_geom(nres, d_out, fz || pipe);
        const int64_t total = g.total, o_first = g.o_first, nblk = g.nblk;
        if (!index_ready || fz || pipe) {
            const int rc = launch_out_index(g, nres, nr, lr, fz, d_span, s);
            if (rc) return rc;
        }
        if (wait_before) SCCG_HIP(hipStreamWaitEvent(s, wait_before, 0));
        if (fz) {
            PROF_LAUNCH(PROF_DC_FORMAT, s, k_format_fused, dim3((unsigned)nblk), dim3(256), 0, s, *fz, nres, total, o_first,
                        (const int32_t*)nr.start, (const int32_t*)nr.len, (const int64_t*)nr.cum, nr.n,
                        (const int32_t*)lr.start, (const int32_t*)lr.len, lr.n, (const int64_t*)d_span, d_out);
            SCCG_HIP(hipGetLastError());
            return 0;
        }
        // (SCCG_FMT_PIPE=1, A/B runs: the resident pipelined grid; measured slower)
        if (pipe) {
            static const int cus = [] {
                int dev = 0, n = 0;
                (void)hipGetDevice(&dev);
                (void)hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev);
                return n > 0 ? n : 256;
            }();
            // resident blocks only (every block walks the same number of tiles: a second generation
            // of blocks would double the time)
            static const int per_cu = [] {
                const char* e = getenv("SCCG_FMT_PIPE_BPC");
                if (e && atoi(e) > 0) return atoi(e);
                int n = 0;
                if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, k_format_pipe, 256, 0) != hipSuccess || n <= 0) n = 4;
                return n;
            }();
            const int64_t g = (int64_t)cus * per_cu < nblk ? (int64_t)cus * per_cu : nblk;
            PROF_LAUNCH(PROF_DC_FORMAT, s, k_format_pipe, dim3((unsigned)g), dim3(256), 0, s, d_dec, nres, total, o_first, nblk,
                        (const int32_t*)nr.start, (const int32_t*)nr.len, (const int64_t*)nr.cum, nr.n,
                        (const int32_t*)lr.start, (const int32_t*)lr.len, lr.n, (const int64_t*)d_span, d_out);
            SCCG_HIP(hipGetLastError());
            return 0;
        }
#define SCCG_FMT_LAUNCH(U, NT)                                                                                       \
    PROF_LAUNCH(PROF_DC_FORMAT, s, (k_format_out<U, NT>), dim3((unsigned)nblk), dim3(256), 0, s, d_dec, nres, total, o_first, \
                (const int32_t*)nr.start, (const int32_t*)nr.len, (const int64_t*)nr.cum, nr.n,                          \
                (const int32_t*)lr.start, (const int32_t*)lr.len, lr.n, (const int64_t*)d_span, d_out)
        const int fu = fmt_u();
        if (fu == 1) { if (fmt_nt) SCCG_FMT_LAUNCH(1, true); else SCCG_FMT_LAUNCH(1, false); }
        else if (fu == 2) { if (fmt_nt) SCCG_FMT_LAUNCH(2, true); else SCCG_FMT_LAUNCH(2, false); }
        else { if (fmt_nt) SCCG_FMT_LAUNCH(4, true); else SCCG_FMT_LAUNCH(4, false); }
#undef SCCG_FMT_LAUNCH
        SCCG_HIP(hipGetLastError());
        return 0;
    }
    if (wait_before) SCCG_HIP(hipStreamWaitEvent(s, wait_before, 0));
    const int64_t nspan = (nres + FSPAN - 1) / FSPAN;
    hipLaunchKernelGGL(k_span_index, dim3(grid_for(2 * (nspan + 1), 256)), dim3(256), 0, s, nres, nspan,
                       (const int32_t*)nr.start, (const int32_t*)nr.len, (const int64_t*)nr.cum, nr.n,
                       (const int32_t*)lr.start, (const int32_t*)lr.len, lr.n, d_span);
    SCCG_HIP(hipGetLastError());
    PROF_LAUNCH(PROF_DC_FORMAT, s, k_format_span, dim3((unsigned)nspan), dim3(256), 0, s, d_dec, nres,
                       (const int32_t*)nr.start, (const int32_t*)nr.len, (const int64_t*)nr.cum, nr.n,
                       (const int32_t*)lr.start, (const int32_t*)lr.len, lr.n, (const int64_t*)d_span, d_out);
    SCCG_HIP(hipGetLastError());
    return 0;
}
