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

// starts = inclusive prefix of deltas (exclusive scan + own delta); runs must be ascending & disjoint
__global__ void k_run_finish(const int64_t* __restrict__ dex, const int64_t* __restrict__ dlt, const int32_t* __restrict__ len,
                             int64_t nr, int32_t* __restrict__ start, int32_t* __restrict__ err) {
    for (int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; r < nr; r += (int64_t)gridDim.x * blockDim.x) {
        const int64_t st = dex[r] + dlt[r];
        const int64_t pst = r ? dex[r - 1] + dlt[r - 1] : INT64_MIN;
        const int64_t pend = r ? pst + len[r - 1] : 0;
        if (st < 0 || st > INT32_MAX || (r && st < pend)) atomicOr(err, 1);
        start[r] = (int32_t)st;
    }
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
                            const int64_t* __restrict__ dlt, const int64_t* __restrict__ contrib, int64_t nref,
                            int32_t* __restrict__ err) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        if (s[i] != '(') continue;
        const int64_t p = dsum[i] + dlt[i];
        if (p < 0 || p + contrib[i] > nref) atomicOr(err, 2);
    }
}

__global__ void k_len_to_i64(const int32_t* __restrict__ len, int64_t n, int64_t* __restrict__ out) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
        out[i] = len[i];
}

constexpr int WPB = 4;
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
    if (i < n) {
        const uint8_t c = s[i];
        const bool inside = lp[i] >= 0 && s[lp[i]] == '(';
        if (c == '(') tok = true;
        else if (!inside) dec[off[i]] = c;   // literals, a stray ')' included
    }
    unsigned long long tm = __ballot(tok);
    while (tm) {
        const int j = __ffsll((long long)tm) - 1;
        tm &= tm - 1;
        const int64_t ij = base + j;
        const int64_t p = dsum[ij] + dlt[ij], l = contrib[ij], o = off[ij];
        for (int64_t q = lane; q < l; q += 64) dec[o + q] = R[p + q];
    }
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
// N positions before j (j inside an N run: those of the run before j included)
__device__ __forceinline__ int64_t n_before(const int32_t* ns, const int32_t* nl, const int64_t* ncum, int64_t nn, int64_t j) {
    const int64_t r = first_run_ending_after(ns, nl, nn, j);
    if (r < nn) return ncum[r] + (ns[r] <= j ? j - ns[r] : 0);
    return nn ? ncum[nn - 1] + nl[nn - 1] : 0;
}
__global__ __launch_bounds__(256) void k_format_span(const uint8_t* __restrict__ dec, int64_t nres,
                                                     const int32_t* __restrict__ ns, const int32_t* __restrict__ nl,
                                                     const int64_t* __restrict__ ncum, int64_t nn,
                                                     const int32_t* __restrict__ ls, const int32_t* __restrict__ ll,
                                                     int64_t nlr, uint8_t* __restrict__ out) {
    __shared__ uint8_t sdec[FSPAN];
    __shared__ uint8_t sout[FSPAN + FSPAN / 50 + 2];
    __shared__ int64_t sd[6];
    const int64_t J0 = (int64_t)blockIdx.x * FSPAN;
    if (J0 >= nres) return;
    const int64_t J1 = J0 + FSPAN < nres ? J0 + FSPAN : nres;
    // one search per block for each run list bounds the runs the span touches: [sd[2], sd[4]] for
    // N, [sd[3], sd[5]] for lowercase; each thread then searches only that range (a span with dense
    // case or N alternation holds up to FSPAN/2 runs, too many to walk forward through)
    if (threadIdx.x == 0) sd[0] = J0 - n_before(ns, nl, ncum, nn, J0);
    if (threadIdx.x == 64) sd[1] = J1 - n_before(ns, nl, ncum, nn, J1);
    if (threadIdx.x == 128) { sd[2] = first_run_ending_after(ns, nl, nn, J0); sd[4] = first_run_ending_after(ns, nl, nn, J1 - 1); }
    if (threadIdx.x == 192) { sd[3] = first_run_ending_after(ls, ll, nlr, J0); sd[5] = first_run_ending_after(ls, ll, nlr, J1 - 1); }
    __syncthreads();
    const int64_t d0 = sd[0], dn = sd[1] - d0;
    for (int64_t i = threadIdx.x; i < dn; i += 256) sdec[i] = dec[d0 + i];
    const int64_t O0 = J0 + J0 / 50;
    const int64_t jl = J1 - 1;
    const int64_t On = jl + jl / 50 + 1 + ((jl % 50 == 49 && jl != nres - 1) ? 1 : 0) - O0;
    __syncthreads();
    const int64_t j0 = J0 + (int64_t)threadIdx.x * FPER;
    if (j0 < J1) {
        // the current N run [n_s, n_e) with the N count before it, the current lowercase run [l_s, l_e)
        int64_t rn = first_run_ending_after(ns, nl, sd[4] < nn ? sd[4] + 1 : nn, j0, sd[2]);
        int64_t rl = first_run_ending_after(ls, ll, sd[5] < nlr ? sd[5] + 1 : nlr, j0, sd[3]);
        int64_t n_s, n_e, n_b, l_s, l_e;
        auto load_n = [&]() {
            if (rn < nn) { n_s = ns[rn]; n_e = n_s + nl[rn]; n_b = ncum[rn]; }
            else { n_s = n_e = INT64_MAX; n_b = nn ? ncum[nn - 1] + nl[nn - 1] : 0; }
        };
        auto load_l = [&]() {
            if (rl < nlr) { l_s = ls[rl]; l_e = l_s + ll[rl]; }
            else l_s = l_e = INT64_MAX;
        };
        load_n();
        load_l();
        for (int64_t j = j0; j < j0 + FPER && j < J1; j++) {
            while (j >= n_e) { rn++; load_n(); }
            while (j >= l_e) { rl++; load_l(); }
            uint8_t c = j >= n_s ? (uint8_t)'N' : sdec[j - n_b - d0];
            if (j >= l_s) c = c_tolower(c);
            const int64_t o = j + j / 50 - O0;
            sout[o] = c;
            if (j % 50 == 49 && j != nres - 1) sout[o + 1] = '\n';
        }
    }
    __syncthreads();
    for (int64_t i = threadIdx.x; i < On; i += 256) out[O0 + i] = sout[i];
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

int dc_last_paren(const uint8_t* d_s, int64_t n, int64_t* d_lp, int64_t* d_partial, hipStream_t s) {
    if (n <= 0) return 0;
    const unsigned g = grid_for(n, 256) > 8192 ? 8192 : grid_for(n, 256);
    hipLaunchKernelGGL(k_paren_pos, dim3(g), dim3(256), 0, s, d_s, n, d_lp);
    SCCG_HIP(hipGetLastError());
    // exclusive max-scan: last parenthesis strictly before i; the inclusive form is not needed
    return dev_excl_max(d_lp, d_lp, n, nullptr, d_partial, s);
}

int dc_parse_runs(const uint8_t* d_s, int64_t n, DcRuns* r, int64_t* d_lp, int64_t* d_flag, int64_t* d_dlt,
                  int64_t* d_partial, int32_t* d_err, int64_t* d_count, hipStream_t s) {
    if (n <= 0) { r->n = 0; return 0; }
    int rc = dc_last_paren(d_s, n, d_lp, d_partial, s);
    if (rc) return rc;
    const unsigned g = grid_for(n, 256) > 8192 ? 8192 : grid_for(n, 256);
    hipLaunchKernelGGL(k_run_items_flag, dim3(g), dim3(256), 0, s, d_s, n, (const int64_t*)d_lp, d_flag, d_err);
    rc = dev_excl_sum(d_flag, d_flag, n, d_count, d_partial, s);
    if (rc) return rc;
    hipLaunchKernelGGL(k_run_items_parse, dim3(g), dim3(256), 0, s, d_s, n, (const int64_t*)d_lp,
                       (const int64_t*)d_flag, d_dlt, r->len, d_err);
    SCCG_HIP(hipGetLastError());
    int64_t nr = 0;
    {
        const RbItem it{d_count, &nr, (int)sizeof nr};
        rc = dev_readback(&it, 1, s);
        if (rc) return rc;
    }
    r->n = nr;
    if (nr == 0) return 0;
    // exclusive sum of deltas into d_flag (free now), then starts
    rc = dev_excl_sum(d_dlt, d_flag, nr, nullptr, d_partial, s);
    if (rc) return rc;
    const unsigned g2 = grid_for(nr, 256) > 8192 ? 8192 : grid_for(nr, 256);
    hipLaunchKernelGGL(k_run_finish, dim3(g2), dim3(256), 0, s, (const int64_t*)d_flag, (const int64_t*)d_dlt,
                       (const int32_t*)r->len, nr, r->start, d_err);
    // cumulative lengths (for N: count of N positions before a run)
    hipLaunchKernelGGL(k_len_to_i64, dim3(g2), dim3(256), 0, s, (const int32_t*)r->len, nr, r->cum);
    SCCG_HIP(hipGetLastError());
    rc = dev_excl_sum(r->cum, r->cum, nr, d_count, d_partial, s);
    if (rc) return rc;
    const RbItem it{d_count, &r->total, (int)sizeof r->total};
    return dev_readback(&it, 1, s);
}

int dc_decode_prepare(const uint8_t* d_s, int64_t n, int64_t* d_lp, int64_t* d_contrib, int64_t* d_dlt, int64_t* d_off,
                      int64_t* d_dsum, int64_t nref, int64_t* d_partial, int32_t* d_err, int64_t* d_total, hipStream_t s) {
    if (n <= 0) {
        SCCG_HIP(hipMemsetAsync(d_total, 0, sizeof(int64_t), s));
        return 0;
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
    hipLaunchKernelGGL(k_tok_check, dim3(g), dim3(256), 0, s, d_s, n, (const int64_t*)d_dsum, (const int64_t*)d_dlt,
                       (const int64_t*)d_contrib, nref, d_err);
    SCCG_HIP(hipGetLastError());
    return 0;
}

int dc_decode_fill(const uint8_t* d_s, int64_t n, const int64_t* d_lp, const int64_t* d_off, const int64_t* d_dsum,
                   const int64_t* d_dlt, const int64_t* d_contrib, const uint8_t* d_R, uint8_t* d_dec, hipStream_t s) {
    if (n <= 0) return 0;
    PROF_LAUNCH(PROF_DC_DECODE, s, k_tok_fill, dim3(grid_for(n, 64 * WPB)), dim3(SCCG_BLOCK), 0, s, d_s, n, d_lp, d_off, d_dsum, d_dlt,
                       d_contrib, d_R, d_dec);
    SCCG_HIP(hipGetLastError());
    return 0;
}

int dc_format(const uint8_t* d_dec, int64_t nres, const DcRuns& nr, const DcRuns& lr, uint8_t* d_out, hipStream_t s) {
    if (nres <= 0) return 0;
    PROF_LAUNCH(PROF_DC_FORMAT, s, k_format_span, dim3(grid_for(nres, FSPAN)), dim3(256), 0, s, d_dec, nres,
                       (const int32_t*)nr.start, (const int32_t*)nr.len, (const int64_t*)nr.cum, nr.n,
                       (const int32_t*)lr.start, (const int32_t*)lr.len, lr.n, d_out);
    SCCG_HIP(hipGetLastError());
    return 0;
}
