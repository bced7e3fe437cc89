// local.hip -- local mode: per-segment match_sequences, the switch state machine, record text.
//
//   segment loop           compression.cpp:372-481
//   match_sequences(r_i, t_i, k, 0, false, i*L)   compression.cpp:36-179 with global=false
//   extend_alignment       compression.cpp:27-34
//
// One wavefront owns one 1000-base segment pair: both segments live in LDS (uppercased on load),
// the reference segment's k-mers go into an LDS open-addressing table (2048 u16 slots), the
// target's "has any candidate" bits are precomputed lane-parallel, and the walk itself is a
// wave-uniform loop that jumps from hit to hit.  Candidates are enumerated 64 table slots at a
// time, extended lane-parallel and reduced with the order-free form of the reference's selection
// loop (tested against the oracle).  Segments are independent, so a launch covers
// every segment; the switch point is found afterwards by a state-machine scan.
#include "internal.h"

namespace {

constexpr int WPB = 4;            // segments (waves) per block
constexpr int SEGB = 1024 + 16;   // LDS bytes per segment string
constexpr int TBITS = 11;         // 2048 table slots
constexpr int TSLOTS = 1 << TBITS;

struct SegLds {
    uint8_t r[SEGB];
    uint8_t t[SEGB];
    uint32_t keys[1000];
    uint32_t table[TSLOTS / 2];   // two u16 slots per word: value = position + 1, 0 = empty
    uint64_t hits[16];            // bit p: target k-mer at p has >= 1 candidate
};

__device__ __forceinline__ uint32_t tab_get(const uint32_t* tab, int slot) {
    return (tab[slot >> 1] >> ((slot & 1) * 16)) & 0xffffu;
}

__device__ __forceinline__ void tab_insert(uint32_t* tab, uint32_t key, uint32_t val) {
    int slot = (int)slot_hash(key, TBITS);
    for (;;) {
        uint32_t* w = &tab[slot >> 1];
        const int sh = (slot & 1) * 16;
        uint32_t old = *w;
        while (((old >> sh) & 0xffffu) == 0) {
            const uint32_t prev = atomicCAS(w, old, old | (val << sh));
            if (prev == old) return;
            old = prev;
        }
        slot = (slot + 1) & (TSLOTS - 1);
    }
}

__device__ __forceinline__ bool bytes_eq(const uint8_t* a, const uint8_t* b, int k) {
    for (int i = 0; i < k; i++) if (a[i] != b[i]) return false;
    return true;
}

template <int K>
__device__ __forceinline__ uint32_t seg_key(const uint8_t* s, int p) {
    return kmer_key(s + p, K);
}

__device__ __forceinline__ uint64_t pick_key(int p, int pme) {
    const int d = p - pme;
    return ((uint64_t)(uint32_t)(d < 0 ? -d : d) << 32) | (uint32_t)p;
}

template <int K>
__global__ __launch_bounds__(SCCG_BLOCK) void k_local_pass(int pass, int upper, const uint8_t* __restrict__ R, int64_t nR,
                                                           const uint8_t* __restrict__ T, int64_t nT, int64_t seg0,
                                                           int64_t seg_end, uint32_t* __restrict__ recs,
                                                           SegStat* __restrict__ stat) {
    __shared__ SegLds lds_all[WPB];
    const int w = wave_in_block(), lane = lane_id();
    const int64_t seg = seg0 + (int64_t)blockIdx.x * WPB + w;
    if (seg >= seg_end) return;
    if (pass == 2 && stat[seg].pass != 0) return;
    SegLds& L = lds_all[w];
    const int64_t base = seg * SEG_L;
    const int nr = (int)((nR - base) < SEG_L ? (nR - base) : SEG_L);
    const int nt = (int)((nT - base) < SEG_L ? (nT - base) : SEG_L);

    // ---- load both segments, uppercased (compression.cpp:369-370, :386-389)
    bool non_n = false;
    for (int i = lane; i < SEGB; i += 64) {
        uint8_t rc = i < nr ? R[base + i] : (uint8_t)0;
        uint8_t tc = i < nt ? T[base + i] : (uint8_t)0;
        if (upper) { rc = c_toupper(rc); tc = c_toupper(tc); }
        L.r[i] = rc;
        L.t[i] = tc;
        non_n |= (i < nt && tc != 'N');
    }
    for (int i = lane; i < TSLOTS / 2; i += 64) L.table[i] = 0;
    if (lane < 16) L.hits[lane] = 0;
    non_n = __ballot(non_n) != 0;
    wave_sync();

    // ---- H: every k-mer of the reference segment (compression.cpp:41-47)
    const int lastr = nr - K;
    {
        const int p0 = lane * 16;
        uint32_t code = 0;
        int lastbad = -1000;
        constexpr uint32_t MASK = (K >= 16) ? 0xffffffffu : ((1u << (2 * K)) - 1u);
        for (int i = 0; i < 16 + K - 1; i++) {
            const int pos = p0 + i;
            const uint8_t c = pos < nr ? L.r[pos] : (uint8_t)0;
            uint32_t b = base2(c);
            if (b > 3) { lastbad = i; b = 0; }
            code = ((code << 2) | b) & MASK;
            const int st = i - (K - 1);
            if (st >= 0) {
                const int p = p0 + st;
                if (p <= lastr) {
                    const uint32_t key = lastbad >= st ? exotic_key(&L.r[p], K) : code;
                    L.keys[p] = key;
                }
            }
        }
    }
    wave_sync();
    for (int p = lane; p <= lastr; p += 64) tab_insert(L.table, L.keys[p], (uint32_t)p + 1);
    wave_sync();

    // ---- hit bits for every target k-mer start (compression.cpp:77 "H.find")
    const int lastk = nt - K;
    {
        const int p0 = lane * 16;
        uint32_t mask16 = 0;
        uint32_t code = 0;
        int lastbad = -1000;
        constexpr uint32_t MASK = (K >= 16) ? 0xffffffffu : ((1u << (2 * K)) - 1u);
        for (int i = 0; i < 16 + K - 1; i++) {
            const int pos = p0 + i;
            const uint8_t c = pos < nt ? L.t[pos] : (uint8_t)0;
            uint32_t b = base2(c);
            if (b > 3) { lastbad = i; b = 0; }
            code = ((code << 2) | b) & MASK;
            const int st = i - (K - 1);
            if (st >= 0) {
                const int p = p0 + st;
                if (p <= lastk && lastr >= 0) {
                    const uint32_t key = lastbad >= st ? exotic_key(&L.t[p], K) : code;
                    int slot = (int)slot_hash(key, TBITS);
                    for (int probes = 0; probes < TSLOTS; probes++) {
                        const uint32_t v = tab_get(L.table, slot);
                        if (!v) break;
                        const int q = (int)v - 1;
                        if (L.keys[q] == key && (key < KEY_EXOTIC || bytes_eq(&L.r[q], &L.t[p], K))) {
                            mask16 |= 1u << st;
                            break;
                        }
                        slot = (slot + 1) & (TSLOTS - 1);
                    }
                }
            }
        }
        reinterpret_cast<uint16_t*>(L.hits)[lane] = (uint16_t)mask16;
    }
    wave_sync();

    // ---- the greedy walk (compression.cpp:64-161), wave-uniform
    uint32_t* out = recs + seg * SEG_REC_CAP;
    int idx = 0, pme = -1, nrec = 0, nmatch = 0, lit = 0, firstp = -1, lastp = -1;
    for (;;) {
        // next target position >= idx with a candidate
        int nxt = -1;
        if (idx <= lastk) {
            for (int wd = idx >> 6; wd < 16; wd++) {
                uint64_t m = L.hits[wd];
                if (wd == (idx >> 6)) m &= ~0ull << (idx & 63);
                if (m) { nxt = wd * 64 + __ffsll((long long)m) - 1; break; }
            }
            if (nxt > lastk) nxt = -1;
        }
        if (nxt < 0) break;
        if (nxt > idx) {
            if (lane == 0) out[nrec] = ((uint32_t)idx << 11) | (uint32_t)(nxt - idx);
            nrec++;
            lit += nxt - idx;
        }
        const uint32_t key = seg_key<K>(L.t, nxt);
        const int h0 = (int)slot_hash(key, TBITS);
        int bl = 0, bcnt = 0;
        bool bhas0 = false;
        uint64_t bkey = ~0ull;
        for (int b0 = 0; b0 < TSLOTS; b0 += 64) {
            const uint32_t v = tab_get(L.table, (h0 + b0 + lane) & (TSLOTS - 1));
            const unsigned long long em = __ballot(v == 0);
            const int fe = first_lane(em);
            if (lane < fe) {
                const int q = (int)v - 1;
                if (L.keys[q] == key && (key < KEY_EXOTIC || bytes_eq(&L.r[q], &L.t[nxt], K))) {
                    int l = K;   // extend_alignment (compression.cpp:27-34)
                    while (q + l < nr && nxt + l < nt && L.r[q + l] == L.t[nxt + l]) ++l;
                    if (l > bl) {
                        bl = l; bcnt = 1; bhas0 = (q == 0); bkey = q ? pick_key(q, pme) : ~0ull;
                    } else if (l == bl) {
                        bcnt++;
                        if (q == 0) bhas0 = true;
                        else { const uint64_t pk = pick_key(q, pme); bkey = pk < bkey ? pk : bkey; }
                    }
                }
            }
            if (em) break;
        }
        const int Lm = wave_max(bl);
        const int cnt = wave_sum(bl == Lm ? bcnt : 0);
        const bool has0 = __ballot(bl == Lm && bhas0) != 0;
        const uint64_t mk = wave_min(bl == Lm ? bkey : ~0ull);
        uint64_t pk;
        if (cnt >= 2 && has0) pk = mk;                 // pn==0 sentinel (compression.cpp:118, :125)
        else {
            const uint64_t k0 = has0 ? pick_key(0, pme) : ~0ull;
            pk = k0 < mk ? k0 : mk;
        }
        const int p = (int)(uint32_t)pk;
        if (lane == 0) out[nrec] = 0x80000000u | ((uint32_t)p << 11) | (uint32_t)Lm;
        nrec++;
        nmatch++;
        if (firstp < 0) firstp = p;
        lastp = p;
        pme = p + Lm - 1;                              // compression.cpp:149
        idx = nxt + Lm;                                // compression.cpp:159
    }
    if (idx < nt) {                                    // compression.cpp:164-167
        if (lane == 0) out[nrec] = ((uint32_t)idx << 11) | (uint32_t)(nt - idx);
        nrec++;
        lit += nt - idx;
    }
    if (lane == 0) {
        SegStat s;
        s.nrec = nrec;
        s.nmatch = nmatch;
        s.lit = lit;
        s.pass = nmatch ? pass : 0;
        s.non_n = pass == 1 ? (int)non_n : stat[seg].non_n;
        s.first_p = firstp;
        s.last_p = lastp;
        s.pad = nt;
        stat[seg] = s;
    }
}

// ---------------------------------------------------------------------------------------------
// switch state machine: state = min(mismatch counter, 5), 6 = switched (absorbing)
// ---------------------------------------------------------------------------------------------
constexpr int FSM_G = 128;   // segments per thread
constexpr int SW = 6;

__device__ __forceinline__ int seg_class(const SegStat& s) {
    // 0 good, 1 success-but-bad (mism++ without check), 2 failed non-N (mism++ + check), 3 failed all-N
    if (s.pass) return (2 * s.lit > s.pad && s.non_n) ? 1 : 0;   // (float)lit/len > 0.5f
    return s.non_n ? 2 : 3;
}

__global__ void k_fsm_chunks(const SegStat* __restrict__ stat, int64_t seg0, int64_t seg_end, int32_t* __restrict__ maps) {
    const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int64_t s0 = seg0 + t * FSM_G;
    if (s0 >= seg_end) return;
    const int64_t s1 = s0 + FSM_G < seg_end ? s0 + FSM_G : seg_end;
    int st[6], at[6];
    for (int i = 0; i < 6; i++) { st[i] = i; at[i] = -1; }
    for (int64_t s = s0; s < s1; s++) {
        const int c = seg_class(stat[s]);
        for (int i = 0; i < 6; i++) {
            if (st[i] == SW) continue;
            if (c == 0 || c == 3) st[i] = 0;
            else if (c == 1) st[i] = st[i] + 1 > 5 ? 5 : st[i] + 1;
            else { if (st[i] + 1 > 4) { st[i] = SW; at[i] = (int)(s - s0); } else st[i]++; }
        }
    }
    for (int i = 0; i < 6; i++) { maps[t * 12 + i] = st[i]; maps[t * 12 + 6 + i] = at[i]; }
}

// ---------------------------------------------------------------------------------------------
// local record text: per segment "(p,l)"/literal records, delta-encoded against the previous
// match token of the whole line (compression.cpp:258-292)
// ---------------------------------------------------------------------------------------------
__global__ void k_seg_lastkey(const SegStat* __restrict__ stat, int64_t iters, int64_t* __restrict__ v) {
    for (int64_t s = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; s < iters; s += (int64_t)gridDim.x * blockDim.x)
        v[s] = (stat[s].pass && stat[s].nmatch) ? s : -1;
}

__device__ __forceinline__ int32_t prev_abs_p(const SegStat* stat, const int64_t* prevseg, int64_t s) {
    const int64_t q = prevseg[s];
    return q >= 0 ? (int32_t)(q * SEG_L + stat[q].last_p) : 0;
}

// one wave per segment: text length
__global__ __launch_bounds__(SCCG_BLOCK) void k_seg_textlen(const SegStat* __restrict__ stat, int64_t iters,
                                                            const uint32_t* __restrict__ recs,
                                                            const int64_t* __restrict__ prevseg,
                                                            int64_t* __restrict__ len) {
    const int64_t s = (int64_t)blockIdx.x * WPB + wave_in_block();
    if (s >= iters) return;
    const int lane = lane_id();
    const SegStat st = stat[s];
    int64_t total = 0;
    if (st.pass) {
        int32_t prev = prev_abs_p(stat, prevseg, s);
        const uint32_t* r = recs + s * SEG_REC_CAP;
        // matches need the previous token's p: do the scan in 64-record batches
        for (int b0 = 0; b0 < st.nrec; b0 += 64) {
            const int i = b0 + lane;
            const uint32_t rec = i < st.nrec ? r[i] : 0;
            const bool is_m = i < st.nrec && (rec >> 31);
            const int32_t pabs = (int32_t)(s * SEG_L) + (int32_t)((rec >> 11) & 0xfffff);
            // previous match p within the batch: last match lane before me
            const unsigned long long mm = __ballot(is_m);
            const unsigned long long before = mm & ((1ull << lane) - 1);
            const int src = before ? 63 - __clzll((long long)before) : -1;
            const int32_t pp = __shfl(pabs, src < 0 ? 0 : src, 64);
            const int32_t my_prev = src >= 0 ? pp : prev;
            int64_t l = 0;
            if (i < st.nrec) {
                if (is_m) l = 3 + ndigits_i32((int32_t)((uint32_t)pabs - (uint32_t)my_prev)) + ndigits_i32((int32_t)(rec & 0x7ff));
                else l = rec & 0x7ff;
            }
            total += wave_sum(l);
            if (mm) prev = __shfl(pabs, 63 - __clzll((long long)mm), 64);
        }
    }
    if (lane == 0) len[s] = total;
}

__global__ __launch_bounds__(SCCG_BLOCK) void k_seg_textwrite(const SegStat* __restrict__ stat, int64_t iters,
                                                              const uint32_t* __restrict__ recs,
                                                              const int64_t* __restrict__ prevseg,
                                                              const int64_t* __restrict__ off,
                                                              const uint8_t* __restrict__ T,
                                                              uint8_t* __restrict__ out) {
    __shared__ int64_t roff[WPB][64];
    const int w = wave_in_block();
    const int64_t s = (int64_t)blockIdx.x * WPB + w;
    if (s >= iters) return;
    const int lane = lane_id();
    const SegStat st = stat[s];
    if (!st.pass) return;
    int32_t prev = prev_abs_p(stat, prevseg, s);
    int64_t o = off[s];
    const uint32_t* r = recs + s * SEG_REC_CAP;
    const int64_t tbase = s * SEG_L;
    for (int b0 = 0; b0 < st.nrec; b0 += 64) {
        const int i = b0 + lane;
        const uint32_t rec = i < st.nrec ? r[i] : 0;
        const bool is_m = i < st.nrec && (rec >> 31);
        const int32_t pabs = (int32_t)(s * SEG_L) + (int32_t)((rec >> 11) & 0xfffff);
        const unsigned long long mm = __ballot(is_m);
        const unsigned long long before = mm & ((1ull << lane) - 1);
        const int src = before ? 63 - __clzll((long long)before) : -1;
        const int32_t pp = __shfl(pabs, src < 0 ? 0 : src, 64);
        const int32_t my_prev = src >= 0 ? pp : prev;
        const int32_t delta = (int32_t)((uint32_t)pabs - (uint32_t)my_prev);
        int64_t l = 0;
        if (i < st.nrec) l = is_m ? 3 + ndigits_i32(delta) + ndigits_i32((int32_t)(rec & 0x7ff)) : (rec & 0x7ff);
        const int64_t incl = wave_incl_add(l);
        const int64_t my_o = o + incl - l;
        if (is_m) {
            uint8_t* d = out + my_o;
            *d++ = '(';
            d += write_i32(d, delta);
            *d++ = ',';
            d += write_i32(d, (int32_t)(rec & 0x7ff));
            *d = ')';
        }
        roff[w][lane] = my_o;
        wave_sync();
        // literal runs: the whole wave copies each one
        unsigned long long lm = __ballot(i < st.nrec && !is_m);
        while (lm) {
            const int j = __ffsll((long long)lm) - 1;
            lm &= lm - 1;
            const uint32_t rj = __shfl(rec, j, 64);
            const int64_t dst = roff[w][j];
            const int start = (int)(rj >> 11), ln = (int)(rj & 0x7ff);
            for (int q = lane; q < ln; q += 64) out[dst + q] = c_toupper(T[tbase + start + q]);
        }
        wave_sync();
        o += __shfl(incl, 63, 64);
        if (mm) prev = __shfl(pabs, 63 - __clzll((long long)mm), 64);
    }
}

__global__ void k_copy_upper(const uint8_t* __restrict__ in, int64_t n, uint8_t* __restrict__ out) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
        out[i] = c_toupper(in[i]);
}

}  // namespace

int launch_local_pass(int k, int pass, int upper, const uint8_t* R, int64_t nR, const uint8_t* T, int64_t nT, int64_t seg0,
                      int64_t seg_end, uint32_t* recs, SegStat* stat, hipStream_t s) {
    if (seg_end <= seg0) return 0;
    const unsigned g = grid_for(seg_end - seg0, WPB);
    if (k == 14)
        PROF_LAUNCH(PROF_LOCAL14, s, k_local_pass<14>, dim3(g), dim3(SCCG_BLOCK), 0, s, pass, upper, R, nR, T, nT, seg0,
                    seg_end, recs, stat);
    else if (k == 10)
        PROF_LAUNCH(PROF_LOCAL10, s, k_local_pass<10>, dim3(g), dim3(SCCG_BLOCK), 0, s, pass, upper, R, nR, T, nT, seg0,
                    seg_end, recs, stat);
    else
        return SCCG_E_UNSUPPORTED;
    SCCG_HIP(hipGetLastError());
    return 0;
}

int64_t fsm_chunks(int64_t iters) { return (iters + FSM_G - 1) / FSM_G; }

int launch_switch_fsm(const SegStat* stat, int64_t seg0, int64_t seg_end, int32_t* d_maps, int32_t* h_maps, int* state,
                      int64_t* switch_seg, hipStream_t s) {
    *switch_seg = -1;
    if (seg_end <= seg0) return 0;
    const int64_t nch = fsm_chunks(seg_end - seg0);
    hipLaunchKernelGGL(k_fsm_chunks, dim3(grid_for(nch, 256)), dim3(256), 0, s, stat, seg0, seg_end, d_maps);
    SCCG_HIP(hipGetLastError());
    SCCG_HIP(hipMemcpyAsync(h_maps, d_maps, (size_t)nch * 12 * sizeof(int32_t), hipMemcpyDeviceToHost, s));
    SCCG_HIP(hipStreamSynchronize(s));
    int st = *state;
    for (int64_t c = 0; c < nch; c++) {
        const int m = h_maps[c * 12 + st];
        if (m == SW) { *switch_seg = seg0 + c * FSM_G + h_maps[c * 12 + 6 + st]; *state = SW; return 0; }
        st = m;
    }
    *state = st;
    return 0;
}

int launch_local_emit(const uint8_t* T, int64_t nT, int64_t iters, const uint32_t* recs, const SegStat* stat,
                      uint8_t* out, int64_t* d_len, int64_t* d_tmp_a, int64_t* d_tmp_b, int64_t* d_partial,
                      hipStream_t s) {
    // d_tmp_a: prev-match segment index, d_tmp_b: per-segment text length -> offsets
    const int64_t lead_len = iters * SEG_L < nT ? iters * SEG_L : nT;
    if (iters > 0) {
        const unsigned g = grid_for(iters, 256) > 4096 ? 4096 : grid_for(iters, 256);
        hipLaunchKernelGGL(k_seg_lastkey, dim3(g), dim3(256), 0, s, stat, iters, d_tmp_a);
        int rc = dev_excl_max(d_tmp_a, d_tmp_a, iters, nullptr, d_partial, s);
        if (rc) return rc;
        hipLaunchKernelGGL(k_seg_textlen, dim3(grid_for(iters, WPB)), dim3(SCCG_BLOCK), 0, s, stat, iters, recs,
                           (const int64_t*)d_tmp_a, d_tmp_b);
        rc = dev_excl_sum(d_tmp_b, d_tmp_b, iters, d_len, d_partial, s);
        if (rc) return rc;
        PROF_LAUNCH(PROF_LOCAL_EMIT, s, k_seg_textwrite, dim3(grid_for(iters, WPB)), dim3(SCCG_BLOCK), 0, s, stat, iters, recs,
                           (const int64_t*)d_tmp_a, (const int64_t*)d_tmp_b, T, out);
        SCCG_HIP(hipGetLastError());
    } else {
        SCCG_HIP(hipMemsetAsync(d_len, 0, sizeof(int64_t), s));
    }
    // leftover target segments (compression.cpp:476-481) go after the segment text
    int64_t seg_text = 0;
    SCCG_HIP(hipMemcpyAsync(&seg_text, d_len, sizeof seg_text, hipMemcpyDeviceToHost, s));
    SCCG_HIP(hipStreamSynchronize(s));
    const int64_t rest = nT - lead_len;
    if (rest > 0) {
        const unsigned g = grid_for(rest, 256) > 8192 ? 8192 : grid_for(rest, 256);
        hipLaunchKernelGGL(k_copy_upper, dim3(g), dim3(256), 0, s, T + lead_len, rest, out + seg_text);
        SCCG_HIP(hipGetLastError());
    }
    const int64_t total = seg_text + (rest > 0 ? rest : 0);
    return dev_set_i64(d_len, 1, {total}, s);
}
