// sccg_api.cpp -- the C ABI (include/sccg.h): context, device buffers, and the compress /
// reconstruct pipelines as sequences of HIP kernel launches on one stream.
//
// Pipeline (compression.cpp:320-582 without the 7z call):
//   find header -> strip target / reference FASTA (ingest.hip)
//   header line, lowercase-run line                            compression.cpp:337-368
//   local segments k=14, then k=10 for the failures (local.hip) compression.cpp:395-452
//   switch state machine                                        compression.cpp:454-473
//   local: ",\n" + segment records + leftover                   compression.cpp:368, :476-481
//   global: N-run line, N erase, windowed walk (walk.hip)       compression.cpp:484-574
// delta_encode (:222-304) is folded into the emitters: each "(p," is written as "(p-p_prev,".
// When the target holds '(' bytes, literals can fool delta_encode's token scan; then the record
// line is written with absolute p (the text before delta_encode) and delta.hip runs that scan.
#include <algorithm>
#include <hip/hip_runtime.h>

#include <fcntl.h>
#include <sys/stat.h>
#include <unistd.h>

#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <future>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "decomp.h"
#include "internal.h"

static thread_local char g_hip_err[512];

int sccg_hip_fail(hipError_t e, const char* what, const char* file, int line) {
    snprintf(g_hip_err, sizeof g_hip_err, "%s:%d: %s -> %s", file, line, what, hipGetErrorString(e));
    return e == hipErrorOutOfMemory ? SCCG_E_NOMEM : SCCG_E_HIP;
}

namespace {

enum Slot {
    B_RFA, B_TFA, B_R, B_T, B_TILE_A, B_TILE_B, B_TILE_FA, B_TILE_FB, B_TILE_LAST, B_TILE_OFF, B_TILE_OFF2, B_TILE_CARRY, B_TILE_BSUM,
    B_SCAL, B_PARTIAL,
    B_RUN_S, B_RUN_E, B_TMP64, B_RUN_SN, B_RUN_EN, B_TMP64N, B_NLINE, B_RECS, B_STAT, B_SEGCLS, B_SEG_A, B_SEG_B, B_RP, B_TP, B_WALK, B_OUT,
    // decompression
    B_D_LP, B_D_FLAG, B_D_DLT, B_D_CONTRIB, B_D_OFF, B_D_DSUM, B_D_LS, B_D_LL, B_D_LC, B_D_NS, B_D_NL, B_D_NC, B_D_DEC, B_D_SPAN, B_D_NLPOS, B_D_LP2, B_D_DLT2, B_PARTIAL2,
    // delta_encode's own token scan (targets holding '(')
    B_DX, B_DELTA,
    // a second FASTA-strip scratch set (the reference strips beside the target, on the side stream)
    B_TILE2_A, B_TILE2_B, B_TILE2_FA, B_TILE2_FB, B_TILE2_LAST, B_TILE2_OFF, B_TILE2_OFF2, B_TILE2_CARRY, B_TILE2_BSUM,
    // fused reconstruction: token table, tokens per record block and their prefix
    B_D_TOK, B_D_BTOK,
    // the target strip's run-event slots (RunSlots) and the run arrays' per-tile scratch
    B_RSLOT, B_RTILE,
    B_COUNT
};
// (the slot numbers tests/test_gpu_oom.py passes in SCCG_TEST_OOM)
static_assert(B_RSLOT == 62 && B_D_DEC == 43 && B_COUNT <= 64, "SCCG_TEST_OOM slot numbers moved");

// Target bases per speculative walk chunk.  Larger chunks mean fewer convergence checks per base,
// smaller ones more chunks in flight: chr1-sized targets (~7.7k chunks of 32 Ki) measured fastest at
// 32 Ki, chromosomes under ~130 Mb and literal-heavy targets at 16 Ki, so the chunk follows the
// target's size in 4 Ki steps between the two (SCCG_WALK_CHUNK overrides it for tuning runs).
constexpr int WALK_CHUNK_MIN = 16384, WALK_CHUNK_MAX = 32768;
constexpr int64_t WALK_CHUNKS_TARGET = 7800;
int walk_chunk(int64_t target_bytes) {
    static const int env = [] {
        const char* e = getenv("SCCG_WALK_CHUNK");
        const int c = e ? atoi(e) : 0;
        return c >= 1024 && c <= (1 << 20) ? c : 0;
    }();
    if (env) return env;
    // (tuning runs: SCCG_WALK_CHUNKS_TARGET / SCCG_WALK_CHUNK_MAX move the size rule)
    static const int64_t target = [] { const char* e = getenv("SCCG_WALK_CHUNKS_TARGET"); const int64_t v = e ? atoll(e) : 0; return v >= 256 ? v : WALK_CHUNKS_TARGET; }();
    static const int64_t cmax = [] { const char* e = getenv("SCCG_WALK_CHUNK_MAX"); const int64_t v = e ? atoll(e) : 0; return v >= WALK_CHUNK_MIN && v <= (1 << 20) ? v : (int64_t)WALK_CHUNK_MAX; }();
    const int64_t c = (target_bytes / target) & ~int64_t(4095);
    return (int)(c < WALK_CHUNK_MIN ? WALK_CHUNK_MIN : c > cmax ? cmax : c);
}
constexpr int DPAD = 4096;   // readable slack after every byte buffer (wide compares, tails)

// SCCG_TEST_OOM: comma-separated slot numbers whose allocation is forced to fail (tests only)
bool oom_slot(int slot) {
    static const uint64_t mask = [] {
        uint64_t m = 0;
        const char* e = getenv("SCCG_TEST_OOM");
        while (e && *e) {
            char* end = nullptr;
            const long v = strtol(e, &end, 10);
            if (end == e) break;
            if (v >= 0 && v < 64) m |= 1ull << v;
            e = *end ? end + 1 : end;
        }
        return m;
    }();
    // each listed slot fails once per process (its first allocation), so a caller's fallback that
    // allocates the same slot later still succeeds
    static std::atomic<uint64_t> failed{0};
    if (slot < 0 || slot >= 64 || !((mask >> slot) & 1)) return false;
    return !((failed.fetch_or(1ull << slot) >> slot) & 1);
}

}  // namespace

// One persistent host thread per context: it runs side work whose launches need host syncs (the
// run lines read their run counts back) while the calling thread drives the main stream.
struct HostWorker {
    std::thread th;
    std::mutex mu;
    std::condition_variable cv;
    std::function<int()> task;
    bool has_task = false, done = true, quit = false;
    int rc = 0;

    void start(int device) {
        th = std::thread([this, device] {
            (void)hipSetDevice(device);
            std::unique_lock<std::mutex> lk(mu);
            for (;;) {
                cv.wait(lk, [this] { return has_task || quit; });
                if (quit) return;
                std::function<int()> f = std::move(task);
                has_task = false;
                lk.unlock();
                const int r = f();
                lk.lock();
                rc = r;
                done = true;
                cv.notify_all();
            }
        });
    }
    void submit(std::function<int()> f) {
        std::lock_guard<std::mutex> lk(mu);
        task = std::move(f);
        has_task = true;
        done = false;
        cv.notify_all();
    }
    int wait() {
        std::unique_lock<std::mutex> lk(mu);
        cv.wait(lk, [this] { return done; });
        return rc;
    }
    void stop() {
        if (!th.joinable()) return;
        {
            std::lock_guard<std::mutex> lk(mu);
            quit = true;
            cv.notify_all();
        }
        th.join();
    }
};

struct sccg_ctx {
    int device = 0;
    HostWorker worker;
    hipStream_t stream = nullptr;
    hipStream_t side = nullptr;       // walk preparation, overlapping the local pass
    hipStream_t side2 = nullptr;      // header + run lines, overlapping the local pass
    hipEvent_t ev_fork = nullptr, ev_fork2 = nullptr, ev_join = nullptr, ev_lines = nullptr, ev_rstrip = nullptr, ev_hdr = nullptr, ev_tstrip = nullptr,
               ev_local = nullptr, ev_probe = nullptr;
    int64_t* h_switch = nullptr;      // pinned: the local pass's switch word, copied behind the pass
    int32_t* h_probe = nullptr;       // pinned: the switch probe's classes and segments (2 PROBE_PAIRS)
    std::string err;
    sccg_stats stats{};
    void* buf[B_COUNT] = {};
    size_t cap[B_COUNT] = {};
    // sccg_compress_files: pinned staging slots (STAGE_THREADS readers x STAGE_SLOTS), one copy
    // stream per input file, allocated on first use
    uint8_t* stage[16] = {};
    hipEvent_t stage_ev[16] = {};
    hipStream_t copy_ref = nullptr, copy_tgt = nullptr;
    hipEvent_t ev_ref_in = nullptr, ev_tgt_in = nullptr;
    void* cls_buf = nullptr;   // local segment classes: buffer the generation tags refer to
    size_t cls_cap = 0;
    int32_t cls_gen = 0;
    bool exact_switch = false;   // SCCG_OPT_EXACT_SWITCH: stats report the reference's first switch

    int fail(int rc, const char* fmt, ...) {
        char tmp[512];
        va_list ap;
        va_start(ap, fmt);
        vsnprintf(tmp, sizeof tmp, fmt, ap);
        va_end(ap);
        err = tmp;
        return rc;
    }
    int hipfail(int rc) {
        err = g_hip_err;
        return rc;
    }
    // device buffer of >= bytes (grown on demand, contents not preserved)
    void* get(int slot, size_t bytes) {
        bytes = (bytes + DPAD + 255) & ~(size_t)255;
        if (cap[slot] >= bytes) return buf[slot];
        if (buf[slot]) { walk_forget_workspace(buf[slot]); (void)hipFree(buf[slot]); }
        buf[slot] = nullptr;
        cap[slot] = 0;
        void* p = nullptr;
        // SCCG_TEST_OOM=<slot>[,<slot>...]: those slots ask for 2^62 bytes, so hipMalloc really
        // fails there (tests of the optional-allocation fallbacks)
        if (oom_slot(slot)) bytes = (size_t)1 << 62;
        if (hipMalloc(&p, bytes) != hipSuccess) {
            // HIP keeps the failure as its last error: clear it, or the next launch check after a
            // caller's fallback would report this out-of-memory
            (void)hipGetLastError();
            return nullptr;
        }
        buf[slot] = p;
        cap[slot] = bytes;
        return p;
    }
};

#define TRY(expr)                                  \
    do {                                           \
        int rc_ = (expr);                          \
        if (rc_) return ctx->hipfail(rc_);         \
    } while (0)
#define HIPTRY(expr)                               \
    do {                                           \
        hipError_t e_ = (expr);                    \
        if (e_ != hipSuccess) return ctx->hipfail(sccg_hip_fail(e_, #expr, __FILE__, __LINE__)); \
    } while (0)
#define GET(T, var, slot, n)                                                            \
    T* var = reinterpret_cast<T*>(ctx->get(slot, (size_t)(n) * sizeof(T)));            \
    if (!var) return ctx->fail(SCCG_E_NOMEM, "device allocation of %zu bytes failed", (size_t)(n) * sizeof(T))

extern "C" {

int sccg_ctx_create(int device, sccg_ctx** out) {
    if (!out) return SCCG_E_INVALID;
    *out = nullptr;
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || n <= 0) return SCCG_E_HIP;
    if (device < 0 || device >= n) return SCCG_E_INVALID;
    if (hipSetDevice(device) != hipSuccess) return SCCG_E_HIP;
    sccg_ctx* c = new sccg_ctx();
    c->device = device;
    // the side stream carries the global walk's critical path (R' sweep -> walk rounds -> text):
    // SCCG_SIDE_PRIORITY=1 (tuning runs) gives it the device's highest stream priority
    int prio_lo = 0, prio_hi = 0;
    (void)hipDeviceGetStreamPriorityRange(&prio_lo, &prio_hi);
    static const bool side_prio = [] { const char* e = getenv("SCCG_SIDE_PRIORITY"); return e && atoi(e) > 0; }();
    if (hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) != hipSuccess ||
        hipStreamCreateWithPriority(&c->side, hipStreamNonBlocking, side_prio ? prio_hi : prio_lo) != hipSuccess ||
        hipStreamCreateWithFlags(&c->side2, hipStreamNonBlocking) != hipSuccess ||
        hipEventCreateWithFlags(&c->ev_fork, hipEventDisableTiming) != hipSuccess ||
        hipEventCreateWithFlags(&c->ev_fork2, hipEventDisableTiming) != hipSuccess ||
        hipEventCreateWithFlags(&c->ev_join, hipEventDisableTiming) != hipSuccess ||
        hipEventCreateWithFlags(&c->ev_lines, hipEventDisableTiming) != hipSuccess ||
        hipEventCreateWithFlags(&c->ev_tstrip, hipEventDisableTiming) != hipSuccess ||
        hipEventCreateWithFlags(&c->ev_rstrip, hipEventDisableTiming) != hipSuccess ||
        hipEventCreateWithFlags(&c->ev_hdr, hipEventDisableTiming) != hipSuccess ||
        hipEventCreateWithFlags(&c->ev_local, hipEventDisableTiming) != hipSuccess ||
        hipEventCreateWithFlags(&c->ev_probe, hipEventDisableTiming) != hipSuccess ||
        hipHostMalloc(reinterpret_cast<void**>(&c->h_probe), 2 * PROBE_PAIRS * sizeof(int32_t), hipHostMallocDefault) != hipSuccess ||
        hipHostMalloc(reinterpret_cast<void**>(&c->h_switch), 64, hipHostMallocDefault) != hipSuccess) {
        delete c;
        return SCCG_E_HIP;
    }
    c->worker.start(device);
    *out = c;
    return SCCG_OK;
}

void sccg_ctx_destroy(sccg_ctx* ctx) {
    if (!ctx) return;
    ctx->worker.stop();
    (void)hipSetDevice(ctx->device);
    (void)hipStreamSynchronize(ctx->stream);
    (void)hipStreamSynchronize(ctx->side);
    (void)hipStreamSynchronize(ctx->side2);
    for (int i = 0; i < B_COUNT; i++)
        if (ctx->buf[i]) { walk_forget_workspace(ctx->buf[i]); (void)hipFree(ctx->buf[i]); }
    (void)hipEventDestroy(ctx->ev_fork);
    (void)hipEventDestroy(ctx->ev_fork2);
    (void)hipEventDestroy(ctx->ev_join);
    (void)hipEventDestroy(ctx->ev_lines);
    (void)hipEventDestroy(ctx->ev_tstrip);
    (void)hipEventDestroy(ctx->ev_rstrip);
    (void)hipEventDestroy(ctx->ev_hdr);
    (void)hipEventDestroy(ctx->ev_local);
    if (ctx->ev_probe) (void)hipEventDestroy(ctx->ev_probe);
    if (ctx->h_probe) (void)hipHostFree(ctx->h_probe);
    if (ctx->h_switch) (void)hipHostFree(ctx->h_switch);
    for (int i = 0; i < 16; i++) {
        if (ctx->stage[i]) (void)hipHostFree(ctx->stage[i]);
        if (ctx->stage_ev[i]) (void)hipEventDestroy(ctx->stage_ev[i]);
    }
    if (ctx->copy_ref) (void)hipStreamDestroy(ctx->copy_ref);
    if (ctx->copy_tgt) (void)hipStreamDestroy(ctx->copy_tgt);
    if (ctx->ev_ref_in) (void)hipEventDestroy(ctx->ev_ref_in);
    if (ctx->ev_tgt_in) (void)hipEventDestroy(ctx->ev_tgt_in);
    (void)hipStreamDestroy(ctx->side);
    (void)hipStreamDestroy(ctx->side2);
    (void)hipStreamDestroy(ctx->stream);
    delete ctx;
}

const char* sccg_last_error(const sccg_ctx* ctx) { return ctx ? ctx->err.c_str() : "null context"; }

int sccg_ctx_set_option(sccg_ctx* ctx, int option, int64_t value) {
    if (!ctx) return SCCG_E_INVALID;
    switch (option) {
        case SCCG_OPT_EXACT_SWITCH: ctx->exact_switch = value != 0; return SCCG_OK;
        default: return SCCG_E_INVALID;
    }
}

int sccg_last_stats(const sccg_ctx* ctx, sccg_stats* out) {
    if (!ctx || !out) return SCCG_E_INVALID;
    *out = ctx->stats;
    return SCCG_OK;
}

void sccg_buf_free(sccg_buf* b) {
    if (!b) return;
    free(b->data);
    b->data = nullptr;
    b->len = 0;
}

void sccg_records_free(sccg_records* r) {
    if (!r) return;
    free(r->kind); free(r->pos); free(r->len); free(r->t);
    memset(r, 0, sizeof *r);
}

size_t sccg_compress_bound(size_t ref_len, size_t tgt_len) {
    (void)ref_len;
    return 12 * tgt_len + 4096;
}

}  // extern "C"

namespace {

int d2h_i64(sccg_ctx* ctx, const int64_t* d, int64_t* h, int n, hipStream_t s = nullptr) {
    const RbItem it{d, h, n * (int)sizeof(int64_t)};
    TRY(dev_readback(&it, 1, s ? s : ctx->stream));
    return 0;
}

// strips one FASTA into `out` (and its filtered copy into out2, when given); returns the kept
// length(s): h_len[0] strip, h_len[1] filter (d_len[0..1] on the device)
// (set 1: the second scratch set, so two strips can run at once; s: stream, default the context's)
int strip(sccg_ctx* ctx, IngestMode mode, const uint8_t* fa, int64_t n, const int64_t* d_hdr, uint8_t* out,
          int64_t* d_len, int32_t* d_flags, int64_t* h_len, FilterMode fmode = FILTER_UPPER, uint8_t* out2 = nullptr,
          int set = 0, hipStream_t s = nullptr, const RunSlots* runs = nullptr) {
    const int64_t ntiles = (n + STRIP_TILE - 1) / STRIP_TILE + 1;
    const int o = set ? B_TILE2_A - B_TILE_A : 0;
    static_assert(B_TILE_BSUM - B_TILE_A == B_TILE2_BSUM - B_TILE2_A, "scratch sets line up");
    IngestScratch sc;
    GET(int64_t, ta, B_TILE_A + o, ntiles);
    GET(int64_t, tb, B_TILE_B + o, ntiles);
    GET(int64_t, tfa, B_TILE_FA + o, ntiles);
    GET(int64_t, tfb, B_TILE_FB + o, ntiles);
    GET(int32_t, tl, B_TILE_LAST + o, ntiles);
    GET(int64_t, to, B_TILE_OFF + o, ntiles);
    GET(int64_t, to2, B_TILE_OFF2 + o, ntiles);
    GET(int32_t, tc, B_TILE_CARRY + o, ntiles);
    // the block sums, then (SCCG_STRIP_KC, default on) the write pass's keep-mask cache: 2 bytes per
    // 64 FASTA bytes, written by the summary and read back instead of classifying plain tiles again
    static const bool kc_on = [] { const char* e = getenv("SCCG_STRIP_KC"); return !e || atoi(e) > 0; }();
    constexpr int64_t KC_AT = 5152;   // (int64s: 1025 x 5 rounded up to 256 bytes)
    GET(int64_t, bs, B_TILE_BSUM + o, kc_on ? KC_AT + ntiles * 16 + (ntiles + 1) / 2 : 1025 * 5);
    sc.tile_a = ta; sc.tile_b = tb; sc.tile_fa = tfa; sc.tile_fb = tfb; sc.tile_last = tl; sc.tile_off = to;
    sc.tile_off2 = to2; sc.tile_carry = tc; sc.block_sums = bs; sc.scalars = nullptr;
    if (kc_on) {
        sc.keep_cache = reinterpret_cast<uint16_t*>(bs + KC_AT);
        sc.keep_flag = reinterpret_cast<int32_t*>(bs + KC_AT + ntiles * 16);
    }
    TRY(launch_fasta_strip(mode, fa, n, d_hdr, out, d_len, d_flags, sc, s ? s : ctx->stream, fmode, out2,
                           out2 ? d_len + 1 : nullptr, runs));
    return h_len ? d2h_i64(ctx, d_len, h_len, out2 ? 2 : 1, s) : 0;   // h_len null: the caller reads d_len later
}

// The target strip's run-event slots (RunSlots) for a FASTA of fa_len bytes, or null (no memory: the
// run lines then take their own passes over T).  The compaction's per-tile scratch comes along.
struct StripRuns {
    RunSlots rs;
    int64_t ntiles = 0;
    int64_t* cs = nullptr;
    int64_t* ce = nullptr;
    int32_t* bev = nullptr;
};
bool strip_runs(sccg_ctx* ctx, int64_t fa_len, StripRuns* out) {
    const int64_t nt = (fa_len + STRIP_TILE - 1) / STRIP_TILE + 1;
    const size_t slots = (size_t)nt * RUN_SLOT;
    uint8_t* a = reinterpret_cast<uint8_t*>(ctx->get(B_RSLOT, 4 * slots * 4 + (size_t)nt * 12 + 64));
    uint8_t* b = reinterpret_cast<uint8_t*>(ctx->get(B_RTILE, (size_t)nt * 20 + 64));
    if (!a || !b) return false;
    RunSlots& r = out->rs;
    r.sl = reinterpret_cast<int32_t*>(a);
    r.el = r.sl + slots;
    r.sn = r.el + slots;
    r.en = r.sn + slots;
    r.rc = reinterpret_cast<uint64_t*>(r.en + slots);
    r.rf = reinterpret_cast<int32_t*>(r.rc + nt);
    r.ovf = r.rf + nt;
    out->ntiles = (fa_len + STRIP_TILE - 1) / STRIP_TILE;   // the tiles the strip writes
    out->cs = reinterpret_cast<int64_t*>(b);
    out->ce = out->cs + nt;
    out->bev = reinterpret_cast<int32_t*>(out->ce + nt);
    return true;
}

// Both run lines of the stripped target (compression.cpp:341-368 lowercase, :495-522 N) in two
// syncs: the run arrays (from the target strip's event slots when it emitted them, else run
// extraction over T for both predicates), one read of both run counts, run text for both, one read
// of both text lengths.  The lowercase line goes to out_lower, the N line to out_n.
int run_lines(sccg_ctx* ctx, const uint8_t* s_in, int64_t n, uint8_t* out_lower, uint8_t** out_n, int64_t* d_sc,
              int64_t* h_lens, hipStream_t s, const StripRuns* sr = nullptr, const int64_t* toff = nullptr,
              const int64_t* d_n = nullptr, const std::function<int(hipStream_t)>& need_input = {}) {
    const int64_t maxruns = n / 2 + 2;
    const int64_t ntiles = (n + INGEST_TILE - 1) / INGEST_TILE + 1;
    const int64_t ntmp = maxruns > ntiles ? maxruns : ntiles;
    GET(int32_t, rs_l, B_RUN_S, maxruns);
    GET(int32_t, re_l, B_RUN_E, maxruns);
    GET(int64_t, tmp_l, B_TMP64, ntmp);
    GET(int32_t, rs_n, B_RUN_SN, maxruns);
    GET(int32_t, re_n, B_RUN_EN, maxruns);
    GET(int64_t, tmp_n, B_TMP64N, ntmp);
    const int64_t npart = ntmp > (sr ? sr->ntiles : 0) ? ntmp : sr->ntiles;
    GET(int64_t, part, B_PARTIAL, 2 * scan_partials_needed(npart) + 16);
    int64_t nruns[3] = {0, 0, 1};
    if (sr) {   // the strip's events; d_sc[4..5] the totals, d_sc[6] <- the overflow flag
        TRY(launch_runs_from_strip(sr->rs, sr->ntiles, toff, d_n, rs_l, re_l, rs_n, re_n, d_sc, sr->cs, sr->ce, sr->bev,
                                   d_sc + 4, part, s));
        int32_t ovf = 0;
        const RbItem it[2] = {{d_sc, nruns, 16}, {sr->rs.ovf, &ovf, 4}};
        TRY(dev_readback(it, 2, s));
        nruns[2] = ovf;
    }
    if (nruns[2]) {   // no slots, or a tile overflowed them: run extraction over T
        if (need_input) TRY(need_input(s));   // (T not written by a lean strip: write it now)
        TRY(launch_runs2(s_in, n, rs_l, re_l, rs_n, re_n, d_sc, tmp_l, tmp_n, part, s));
        TRY(d2h_i64(ctx, d_sc, nruns, 2, s));
    }
    TRY(launch_run_text(rs_l, re_l, nruns[0], n, out_lower, d_sc + 2, tmp_l, part, s));
    GET(uint8_t, nline, B_NLINE, 24 * nruns[1] + 16);   // <= 23 text bytes per run
    *out_n = nline;
    TRY(launch_run_text(rs_n, re_n, nruns[1], n, nline, d_sc + 3, tmp_n, part, s));
    return d2h_i64(ctx, d_sc + 2, h_lens, 2, s);
}

// delta_encode's token scan over an absolute-p record line X (delta.hip)
int paren_delta(sccg_ctx* ctx, const uint8_t* X, int64_t n, uint8_t* out, int64_t cap, int64_t* len, bool* stoi_fail) {
    void* ws = ctx->get(B_DELTA, delta_workspace_bytes(n));
    if (!ws) return ctx->fail(SCCG_E_NOMEM, "delta workspace of %zu bytes", delta_workspace_bytes(n));
    TRY(delta_encode_dev(X, n, out, cap, len, stoi_fail, ws, ctx->stream));
    return 0;
}

// the parameter sets the kernels are built for (sccg.h, sccg_params)
int check_params(sccg_ctx* ctx, const sccg_params& P) {
    if (P.m < 0 || 2 * P.m + 1 > 256)
        return ctx->fail(SCCG_E_UNSUPPORTED, "m = %d: the global walk's window takes 0 <= m <= 127", P.m);
    if (P.local) {
        if (P.k != 14 || P.k2 != 10 || P.L != SEG_L || P.T1 != 0.5f || P.T2 != 4)
            return ctx->fail(SCCG_E_UNSUPPORTED, "local = 1 takes the reference's k = 14, k2 = 10, L = 1000, T1 = 0.5, T2 = 4 "
                                                 "(use local = 0 for other k)");
    } else if (P.k < 1 || P.k > 32) {
        return ctx->fail(SCCG_E_UNSUPPORTED, "k = %d: the global walk takes 1 <= k <= 32", P.k);
    }
    return 0;
}

// Host-side readiness of the two FASTA texts (sccg_compress_files): each hook blocks until that
// file's bytes are all queued on a copy stream and returns an event behind them; the pipeline waits
// on it right before the first kernel that reads the file, so the reference's strip (and the R'
// sweep behind it) run while the target is still being read.
struct InputReady {
    int (*ref)(void* user, hipEvent_t* ev);
    int (*tgt)(void* user, hipEvent_t* ev);
    void* user;
};

int compress_device_impl(sccg_ctx* ctx, const sccg_params& P, const uint8_t* rfa, int64_t rn, const uint8_t* tfa,
                         int64_t tn, uint8_t* out, int64_t out_cap, int64_t* out_len, const InputReady* rdy = nullptr) {
    hipStream_t s = ctx->stream;
    if (const int rc = check_params(ctx, P)) return rc;
    // local = 0: no local pass, the global pass from the start (compression.cpp:378, :484)
    const bool force_global = !P.local;
    const int kg = P.k, mg = P.m;   // the global call's k and m (compression.cpp:561)
    sccg_stats st{};
    st.switch_segment = -1;
    // SCCG_DEBUG: host-side phase clock (synchronises at every mark, diagnostics only)
    const bool dbg = getenv("SCCG_DEBUG") != nullptr;
    auto t_last = std::chrono::steady_clock::now();
    auto mark = [&](const char* what) {
        if (!dbg) return;
        (void)hipStreamSynchronize(s);
        const auto t = std::chrono::steady_clock::now();
        fprintf(stderr, "[phase] %-14s %8.3f ms\n", what, std::chrono::duration<double, std::milli>(t - t_last).count());
        t_last = t;
    };
    GET(int64_t, sc, B_SCAL, 64);
    GET(uint8_t, T, B_T, tn + 64);
    GET(uint8_t, R, B_R, rn + 64);
    // N-erased, uppercased copies for the global pass (compression.cpp:523-524, :556-557), written
    // by the same ingest pass (the local pass may end up not needing them)
    GET(uint8_t, Tp, B_TP, tn + 64);
    GET(uint8_t, Rp, B_RP, rn + 64);
    // Lean strips (round 6): the unfiltered stripped copies T and R are read only by the local pass
    // (and by the run-line fallback when a tile overflows its run-event slots).  When the switch
    // probe decides the mode (or there is no local pass, local = 0), the strips write only T' and
    // R'; the probe gathers its segments of T and R from the FASTA (k_strip_gather), and a pair it
    // leaves local gets T and R from a second write pass (launch_strip_rewrite) before its pass.
    const int64_t iters_max = ((rn < tn ? rn : tn) + SEG_L - 1) / SEG_L;   // FASTA lengths bound the sequences'
    static const bool lean_on = [] { const char* e = getenv("SCCG_LEAN_STRIP"); return !e || atoi(e) != 0; }();
    const bool probe_mode = !force_global && !ctx->exact_switch && iters_max > 0 && local_probe_applies(iters_max);
    const bool lean_R = lean_on && (probe_mode || force_global);
    int32_t* d_flags = reinterpret_cast<int32_t*>(sc + 32);
    HIPTRY(hipMemsetAsync(d_flags, 0, sizeof(int32_t), s));
    // local pass control {0, early-exit bound, switch segment, 0}: INT32_MAX = none yet
    TRY(dev_set_i64(sc + 20, 2, {(int64_t)INT32_MAX << 32, (int64_t)INT32_MAX}, s));

    // ---- ingest (compression.cpp:181-220)
    // header search and both strips run back to back; one sync reads every length (sc[0..9])
    // the reference strips on the side stream beside the target's header search + strip
    global_prepare_reset();
    // The target's header search (one block) goes first when both inputs are resident: queued
    // behind the reference strip's grid it waited ~85 us for issue slots on the chr1 pair, and the
    // target strip -- on the walk's critical path -- waits for it.
    HIPTRY(hipEventRecord(ctx->ev_fork, s));   // (the side stream forks before the search: no wait on it)
    if (!rdy) TRY(launch_find_header(tfa, tn, sc, s));
    HIPTRY(hipStreamWaitEvent(ctx->side, ctx->ev_fork, 0));
    if (rdy) {
        hipEvent_t e = nullptr;
        if (const int rc = rdy->ref(rdy->user, &e)) return rc;
        HIPTRY(hipStreamWaitEvent(ctx->side, e, 0));
    }
    TRY(strip(ctx, INGEST_REF, rfa, rn, nullptr, lean_R ? nullptr : R, sc + 7, nullptr, nullptr, FILTER_DROP_N_UPPER, Rp, 1,
              ctx->side));
    HIPTRY(hipEventRecord(ctx->ev_rstrip, ctx->side));
    if (rdy) {
        hipEvent_t e = nullptr;
        if (const int rc = rdy->tgt(rdy->user, &e)) return rc;
        HIPTRY(hipStreamWaitEvent(s, e, 0));
        TRY(launch_find_header(tfa, tn, sc, s));
    }
    HIPTRY(hipEventRecord(ctx->ev_hdr, s));
    // the target strip also emits both run lines' boundaries (RunSlots): no extra passes over T
    StripRuns sruns;
    const bool have_runs = strip_runs(ctx, tn, &sruns);
    if (have_runs) HIPTRY(hipMemsetAsync(sruns.rs.ovf, 0, sizeof(int32_t), s));
    const bool lean_T = lean_R && have_runs;   // (without run-event slots the run lines read T)
    TRY(strip(ctx, INGEST_TGT, tfa, tn, sc, lean_T ? nullptr : T, sc + 2, d_flags, nullptr, FILTER_DROP_N_UPPER, Tp, 0,
              nullptr, have_runs ? &sruns.rs : nullptr));
    // T and R written after all (a pair the probe leaves local, or a run-slot overflow), from the
    // strips' tile offsets (scratch sets 0 and 1); each at most once per stream that needs it
    auto rewrite = [&](IngestMode mode, hipStream_t st) -> int {
        const int o = mode == INGEST_REF ? B_TILE2_A - B_TILE_A : 0;
        IngestScratch isc{};
        isc.tile_off = reinterpret_cast<int64_t*>(ctx->buf[B_TILE_OFF + o]);
        isc.tile_off2 = reinterpret_cast<int64_t*>(ctx->buf[B_TILE_OFF2 + o]);
        isc.tile_carry = reinterpret_cast<int32_t*>(ctx->buf[B_TILE_CARRY + o]);
        return mode == INGEST_REF ? launch_strip_rewrite(INGEST_REF, rfa, rn, nullptr, R, isc, st)
                                  : launch_strip_rewrite(INGEST_TGT, tfa, tn, sc, T, isc, st);
    };
    // ---- header + lowercase line (compression.cpp:337-368) and the N line: side2, driven by the
    //      context's host worker (its launches wait on run counts).  They need only T, so they are
    //      queued right behind the target's strip -- ahead of the local pass and the walk, which
    //      would otherwise share the GPU with these bandwidth-heavy passes.
    HIPTRY(hipEventRecord(ctx->ev_tstrip, s));
    hipStream_t s3 = ctx->side2;
    HIPTRY(hipStreamWaitEvent(s3, ctx->ev_tstrip, 0));
    uint8_t* nline = nullptr;
    int64_t rl_len[2] = {0, 0};
    // the worker's first readback (header range, |T|, |T'|, the '(' flag, |R|, |R'|) is this
    // thread's too
    int64_t h4[4] = {0, 0, 0, 0}, lr[2] = {0, 0};
    HIPTRY(hipStreamWaitEvent(s3, ctx->ev_rstrip, 0));
    int32_t flags = 0;
    std::promise<int> lens_read;
    std::future<int> lens = lens_read.get_future();
    ctx->worker.submit([&, s3]() -> int {
        {
            const RbItem it[3] = {{sc, h4, (int)sizeof h4}, {d_flags, &flags, (int)sizeof flags}, {sc + 7, lr, (int)sizeof lr}};
            const int rc = dev_readback(it, 3, s3);
            lens_read.set_value(rc);
            if (rc) return ctx->hipfail(rc);
        }
        const bool hh = h4[0] < tn;
        const int64_t hl = hh ? h4[1] - h4[0] : 0;
        // (this thread reports both conditions; the worker only must not write)
        if (h4[2] >= INT32_MAX - 8 || out_cap < hl + 1 + 11 * h4[2] + 64) return 0;
        if (hh) {
            HIPTRY(hipMemcpyAsync(out, tfa + h4[0], (size_t)hl, hipMemcpyDeviceToDevice, s3));
            TRY(dev_put_bytes(out + hl, "\n", 1, s3));
        }
        // both run lines now (the N line is kept aside until the mode is known)
        TRY(run_lines(ctx, T, h4[2], out + (hh ? hl + 1 : 0), &nline, sc + 10, rl_len, s3, have_runs ? &sruns : nullptr,
                      reinterpret_cast<const int64_t*>(ctx->buf[B_TILE_OFF]), sc + 2,
                      lean_T ? std::function<int(hipStream_t)>([&](hipStream_t st) { return rewrite(INGEST_TGT, st); })
                             : std::function<int(hipStream_t)>()));
        HIPTRY(hipEventRecord(ctx->ev_lines, s3));
        return 0;
    });
    struct WorkerJoin {   // every exit path waits for the side work (it captures this frame)
        HostWorker* w;
        bool joined = false;
        int join() {
            if (joined) return 0;
            joined = true;
            return w->wait();
        }
        ~WorkerJoin() { join(); }
    } lines{&ctx->worker};
    // The walk's R'-only preparation (anchor samples, positions of the target's first k-mer read off
    // its FASTA) starts on the side stream as soon as R' exists, beside the target's strip.
    // The walk workspace is sized by the FASTA lengths (>= |R'|, |T'|), so the early sweep needs no
    // host read of |R'| (it reads it on the device) and the walk reuses the same carve.
    const size_t wsb = walk_workspace_bytes(rn, tn, kg, walk_chunk(tn));
    if (rn < INT32_MAX - 8 && tn < INT32_MAX - 8) {
        HIPTRY(hipStreamWaitEvent(ctx->side, ctx->ev_hdr, 0));
        void* ws_early = ctx->get(B_WALK, wsb);
        if (!ws_early) return ctx->fail(SCCG_E_NOMEM, "walk workspace of %zu bytes", wsb);
        TRY(global_sweep_early(Rp, rn, sc + 8, tfa, tn, sc, kg, mg, walk_chunk(tn), ws_early, wsb, ctx->side));
    }
    HIPTRY(hipStreamWaitEvent(s, ctx->ev_rstrip, 0));
    // ---- fork.  The local pass (compression.cpp:372-474, main stream) is latency-bound; the
    //      global walk's input-only preparation (side stream) and the header + run lines (side2)
    //      only read T/R/T'/R', so they run beside it.  The local pass reads |R|, |T| from device
    //      memory and is queued before the host reads the lengths back (on side2).
    hipStream_t s2 = ctx->side;
    HIPTRY(hipEventRecord(ctx->ev_fork, s));
    HIPTRY(hipStreamWaitEvent(s2, ctx->ev_fork, 0));
    GET(uint32_t, recs, B_RECS, (iters_max > 0 ? iters_max : 1) * SEG_REC_CAP);
    GET(SegStat, stat, B_STAT, iters_max > 0 ? iters_max : 1);
    // (the switch probe's output after the classes: 2 PROBE_PAIRS words)
    // (after the classes: the switch probe's output (2 PROBE_PAIRS words), its segment list
    // (PROBE_PAIRS) and the gathered T and R segments (2 PROBE_PAIRS * SEG_GATHER_B bytes))
    constexpr int64_t PROBE_WORDS = 3 * PROBE_PAIRS + 2 * PROBE_PAIRS * SEG_GATHER_B / 4;
    GET(int32_t, cls, B_SEGCLS, (iters_max > 0 ? iters_max : 1) + PROBE_WORDS + 64);
    int32_t* probe_out = cls + (((iters_max > 0 ? iters_max : 1) + 63) & ~int64_t(63));
    int32_t* probe_segs = probe_out + 2 * PROBE_PAIRS;
    uint8_t* probe_gT = reinterpret_cast<uint8_t*>(probe_segs + PROBE_PAIRS);
    uint8_t* probe_gR = probe_gT + PROBE_PAIRS * SEG_GATHER_B;
    int32_t* ctl = reinterpret_cast<int32_t*>(sc + 20);   // {0, bound, switch, 0}
    // Where the local pass goes.  It fills every CU while it runs (LDS and VGPRs), but only the final
    // record text needs it; the global walk (side stream) is the critical path of a switching pair.
    //   0: right after both strips (beside the R' sweep);  1: behind the walk's preparation (the
    //   first-step statistics);  2: behind walk round 1 (SCCG_LOCAL_ORDER, tuning runs)
    static const int local_order = [] { const char* e = getenv("SCCG_LOCAL_ORDER"); const int v = e ? atoi(e) : 0; return v >= 0 && v <= 2 ? v : 0; }();
    bool local_launched = false;
    // The switch probe (default; not with SCCG_OPT_EXACT_SWITCH): a few runs of segments spread over
    // the pair are classified first (local.hip k_local_probe); one complete switch window among them
    // decides the pair global (a switching pair's record file does not depend on where it switched,
    // compression.cpp:462-473, :484-574), so the in-order pass is launched only when they hold none.
    // The host reads the probe's 1 KiB back behind the walk's first rounds (decide_probe).
    bool probe_pending = false;
    auto launch_inorder = [&]() -> int {
        if (cls != ctx->cls_buf || ctx->cap[B_SEGCLS] != ctx->cls_cap || ctx->cls_gen >= (1 << 28)) {
            // a new buffer (or tags about to wrap): zero it once, so no stale tag can match
            HIPTRY(hipMemsetAsync(cls, 0, ctx->cap[B_SEGCLS], s));
            ctx->cls_buf = cls;
            ctx->cls_cap = ctx->cap[B_SEGCLS];
            ctx->cls_gen = 0;
        }
        const int32_t gen = ++ctx->cls_gen;
        // one launch over every segment; segments past a detected switch are never started
        TRY(launch_local_all(R, sc + 7, T, sc + 2, iters_max, recs, stat, cls, gen, ctl, s));
        return 0;
    };
    auto launch_local = [&](hipStream_t after) -> int {
        if (local_launched) return 0;
        local_launched = true;
        if (after) {
            HIPTRY(hipEventRecord(ctx->ev_fork2, after));
            HIPTRY(hipStreamWaitEvent(s, ctx->ev_fork2, 0));
        }
        if (iters_max > 0 && !force_global) {
            if (probe_mode) {
                // the probed segments of T and R, from the FASTA when the strips did not write them
                TRY(launch_probe_segs(sc + 7, sc + 2, probe_segs, s));
                if (lean_T) {
                    TRY(launch_strip_gather(INGEST_TGT, tfa, tn, sc, reinterpret_cast<const int64_t*>(ctx->buf[B_TILE_OFF]),
                                            reinterpret_cast<const int32_t*>(ctx->buf[B_TILE_CARRY]), sc + 2, probe_segs,
                                            PROBE_PAIRS, probe_gT, s));
                } else {
                    TRY(launch_segment_copy(T, sc + 2, probe_segs, PROBE_PAIRS, probe_gT, s));
                }
                if (lean_R) {
                    TRY(launch_strip_gather(INGEST_REF, rfa, rn, nullptr, reinterpret_cast<const int64_t*>(ctx->buf[B_TILE2_OFF]),
                                            reinterpret_cast<const int32_t*>(ctx->buf[B_TILE2_CARRY]), sc + 7, probe_segs,
                                            PROBE_PAIRS, probe_gR, s));
                } else {
                    TRY(launch_segment_copy(R, sc + 7, probe_segs, PROBE_PAIRS, probe_gR, s));
                }
                TRY(launch_local_probe(probe_gR, sc + 7, probe_gT, sc + 2, probe_segs, probe_out, s));
                HIPTRY(hipMemcpyAsync(ctx->h_probe, probe_out, 2 * PROBE_PAIRS * sizeof(int32_t), hipMemcpyDeviceToHost, s));
                HIPTRY(hipEventRecord(ctx->ev_probe, s));
                probe_pending = true;
            } else {
                TRY(launch_inorder());
            }
        }
        return 0;
    };
    if (local_order == 0) TRY(launch_local(nullptr));
    TRY(lens.get());
    const int64_t hdr[2] = {h4[0], h4[1]}, lt[2] = {h4[2], h4[3]};
    const int64_t nT = lt[0], nR = lr[0];
    if (nT >= INT32_MAX - 8 || nR >= INT32_MAX - 8)
        return ctx->fail(SCCG_E_UNSUPPORTED, "sequence longer than the reference's int positions allow");
    // a '(' among the target bytes can reach the record line as a literal (see delta.hip)
    const bool paren = (flags & 1) != 0;
    bool stoi_fail = false;
    st.target_bases = nT;
    st.reference_bases = nR;
    st.walk_reference_bases = lr[1];
    mark("ingest");
    const bool has_hdr = hdr[0] < tn;
    const int64_t hlen = has_hdr ? hdr[1] - hdr[0] : 0;
    if (out_cap < hlen + 1 + 11 * nT + 64) return ctx->fail(SCCG_E_INVALID, "output capacity too small");

    const int64_t nRs = (nR + SEG_L - 1) / SEG_L, nTs = (nT + SEG_L - 1) / SEG_L;
    const int64_t iters = nRs < nTs ? nRs : nTs;   // segments the local pass took (its device count)
    int64_t sw = -1;

    // ---- the global walk's preparation, side stream (wasted only if the pass stays local)
    const int64_t np[2] = {lt[1], lr[1]};
    void* ws = ctx->get(B_WALK, wsb);
    if (!ws) return ctx->fail(SCCG_E_NOMEM, "walk workspace of %zu bytes", wsb);
    TRY(global_prepare(Rp, np[1], Tp, np[0], kg, mg, walk_chunk(tn), ws, wsb, s2));
    HIPTRY(hipEventRecord(ctx->ev_join, s2));
    if (local_order == 1 || iters <= 0 || force_global) TRY(launch_local(s2));

    int64_t pos = 0;
    auto join_lines = [&](hipStream_t on) -> int {   // the lowercase line's end, `on` ordered after it
        TRY(lines.join());
        HIPTRY(hipStreamWaitEvent(on, ctx->ev_lines, 0));
        pos = (has_hdr ? hlen + 1 : 0) + rl_len[0];
        return 0;
    };

    // ---- the switch point (compression.cpp:417-481), read once the local pass is done
    bool sw_known = iters <= 0 || force_global;
    auto local_tail = [&]() -> int {   // the switch word behind the local pass, and its event
        if (iters > 0 && !force_global) HIPTRY(hipMemcpyAsync(ctx->h_switch, sc + 21, sizeof(int64_t), hipMemcpyDeviceToHost, s));
        HIPTRY(hipEventRecord(ctx->ev_local, s));
        return 0;
    };
    // the probe's verdict: a window decides the mode (no in-order pass at all), none queues the pass
    auto decide_probe = [&]() -> int {
        if (!probe_pending) return 0;
        probe_pending = false;
        HIPTRY(hipEventSynchronize(ctx->ev_probe));
        const int32_t w = local_probe_window(ctx->h_probe);
        if (w >= 0) {
            sw = w;
            sw_known = true;
            HIPTRY(hipEventRecord(ctx->ev_local, s));
            return 0;
        }
        if (lean_T) TRY(rewrite(INGEST_TGT, s));   // (the local pass reads T and R)
        if (lean_R) TRY(rewrite(INGEST_REF, s));
        TRY(launch_inorder());
        return local_tail();
    };
    auto read_switch = [&]() -> int {
        TRY(decide_probe());
        if (sw_known) return 0;
        HIPTRY(hipEventSynchronize(ctx->ev_local));
        const int64_t h_sw = *ctx->h_switch;   // ctl[2] | ctl[3] << 32
        sw = h_sw >= INT32_MAX ? -1 : h_sw;
        sw_known = true;
        return 0;
    };
    if (local_launched && !probe_pending) TRY(local_tail());
    auto ensure_local = [&](hipStream_t after) -> int {   // (order 2 when the walk never queued round 1)
        if (local_launched) return 0;
        TRY(launch_local(after));
        return probe_pending ? 0 : local_tail();
    };

    // ---- global (compression.cpp:484-574), speculatively: the walk runs on the side stream right
    //      behind its preparation, beside the local pass, and is abandoned if the pass finds no
    //      switch (checked after every walk round, and before any record text is written).
    bool global_done = false;
    int64_t g_rlen = 0;
    uint8_t* X = nullptr;
    WalkResult wr{};
    if (iters > 0 || force_global) {
        struct Late {
            std::function<int(uint8_t**)> f;
            std::function<int()> poll;
            static int call(void* u, uint8_t** o) { return static_cast<Late*>(u)->f(o); }
            static int abandon(void* u) { return static_cast<Late*>(u)->poll(); }
            std::function<int(hipStream_t)> r1;
            static int round1(void* u, hipStream_t st) { return static_cast<Late*>(u)->r1(st); }
        } late{[&](uint8_t** o) -> int {
                   TRY(ensure_local(s2));
                   TRY(read_switch());
                   if (sw < 0 && !force_global) return WALK_ABANDONED;
                   TRY(join_lines(s2));
                   const int64_t nlen = rl_len[1];
                   TRY(dev_put_framed(out + pos, nline, nlen, '\n', '\n', s2));   // "\n" + N line + "\n"
                   pos += nlen + 2;
                   X = out + pos;
                   if (paren) {
                       GET(uint8_t, xb, B_DX, out_cap - pos);
                       X = xb;
                   }
                   *o = X;
                   return 0;
               },
               [&]() -> int {
                   if (force_global || !local_launched) return 0;
                   if (decide_probe()) return 0;   // (the resolve step reports the error)
                   if (!sw_known && hipEventQuery(ctx->ev_local) != hipSuccess) return 0;   // pass still running
                   if (read_switch()) return 0;   // the resolve step reports the error
                   return sw < 0;
               },
               [&](hipStream_t st) -> int {
                   // (the probe's verdict once the walk's first rounds are queued: the in-order pass,
                   // when needed, then runs beside them)
                   TRY(local_order == 2 ? ensure_local(st) : 0);
                   return decide_probe();
               }};
        const EmitTarget target{&Late::call, &late, &Late::abandon, &Late::round1};
        const int rc = global_match_and_emit(Rp, np[1], Tp, np[0], kg, mg, walk_chunk(tn), ws, wsb, nullptr, &g_rlen, &wr,
                                             s2, paren, &target, /*keep_flat=*/false);
        if (rc != WALK_ABANDONED) {
            TRY(rc);
            if (!X) return ctx->fail(SCCG_E_INTERNAL, "record text position never resolved");
            global_done = true;
        }
    }
    TRY(ensure_local(s2));
    HIPTRY(hipEventRecord(ctx->ev_join, s2));   // all side work (preparation, walk) before anything reuses it
    HIPTRY(hipStreamWaitEvent(s, ctx->ev_join, 0));
    TRY(read_switch());
    st.switch_segment = sw;
    mark("local");
    if (!global_done) {
        if (sw >= 0 || force_global) return ctx->fail(SCCG_E_INTERNAL, "switch found but the global walk was abandoned");
        global_prepare_reset();
        TRY(join_lines(s));
        // ---- local: "\n,\n" + records + leftover segments
        TRY(dev_put_bytes(out + pos, "\n,\n", 3, s));
        pos += 3;
        GET(int64_t, sa, B_SEG_A, iters + 1);
        GET(int64_t, sb, B_SEG_B, iters + 1);
        GET(int64_t, part, B_PARTIAL, scan_partials_needed(iters + 1) + 16);
        uint8_t* XL = out + pos;
        if (paren) {
            GET(uint8_t, xb, B_DX, out_cap - pos);
            XL = xb;
        }
        TRY(launch_local_proven(R, nR, T, nT, iters, recs, stat, s));   // records of the segments proved class 0
        TRY(launch_local_emit(T, nT, iters, recs, stat, XL, sc + 5, sa, sb, part, s, paren));
        int64_t rlen = 0;
        TRY(d2h_i64(ctx, sc + 5, &rlen, 1));
        if (paren) TRY(paren_delta(ctx, XL, rlen, out + pos, out_cap - pos, &rlen, &stoi_fail));
        // statistics: match tokens / literal bases of the record line
        std::vector<SegStat> hs((size_t)(iters > 0 ? iters : 0));
        if (iters > 0) {
            HIPTRY(hipMemcpyAsync(hs.data(), stat, (size_t)iters * sizeof(SegStat), hipMemcpyDeviceToHost, s));
            HIPTRY(hipStreamSynchronize(s));
        }
        int64_t nm = 0, lit = 0;
        for (auto& x : hs) if (x.pass) { nm += x.nmatch; lit += x.lit; }
        const int64_t lead = iters * SEG_L < nT ? iters * SEG_L : nT;
        st.n_matches = nm;
        st.literal_bases = lit + (nT - lead);
        pos += rlen;
    } else {
        st.mode_global = 1;
        int64_t rlen = g_rlen;
        if (paren) TRY(paren_delta(ctx, X, rlen, out + pos, out_cap - pos, &rlen, &stoi_fail));
        st.n_matches = wr.n_matches;
        st.walk_rounds = wr.rounds;
        st.walk_chunks = wr.chunks;
        st.walk_chains = wr.chains;
        pos += rlen;
        mark("global_walk");
    }
    HIPTRY(hipStreamSynchronize(s));
    st.record_bytes = pos;
    ctx->stats = st;
    *out_len = pos;
    if (stoi_fail)   // compression.cpp:279 throws: the file keeps the absolute text, main returns 1
        return ctx->fail(SCCG_E_DELTA_STOI, "delta_encode: stoi fails on a token of the record line");
    return SCCG_OK;
}


// -------------------------------------------------------------------------------------------
// FASTA files -> compressed_genome.txt (read_genomes_from_files, compression.cpp:181-220, up to the
// record file of :329, without 7z).  STAGE_THREADS host threads read both files in STAGE_PIECE
// pieces with pread() into pinned slots (two per thread), and each piece goes to HBM on its file's
// copy stream as soon as it is read; the reference is read first, so its strip and the R' sweep
// run on the GPU while the target is still being read.  The record text comes back through the
// same pinned slots, a piece at a time, and is written as it arrives.
// -------------------------------------------------------------------------------------------
constexpr int STAGE_THREADS = 4, STAGE_SLOTS = 2;
constexpr size_t STAGE_PIECE = (size_t)16 << 20;
static_assert(STAGE_THREADS * STAGE_SLOTS <= 16, "sccg_ctx::stage");

int staging_init(sccg_ctx* ctx) {
    // idempotent piece by piece: a call after a partial failure completes what is missing instead of
    // allocating (and leaking) the slots and events again
    for (int i = 0; i < STAGE_THREADS * STAGE_SLOTS; i++) {
        if (!ctx->stage[i]) HIPTRY(hipHostMalloc(reinterpret_cast<void**>(&ctx->stage[i]), STAGE_PIECE, hipHostMallocDefault));
        if (!ctx->stage_ev[i]) HIPTRY(hipEventCreateWithFlags(&ctx->stage_ev[i], hipEventDisableTiming));
    }
    if (!ctx->ev_ref_in) HIPTRY(hipEventCreateWithFlags(&ctx->ev_ref_in, hipEventDisableTiming));
    if (!ctx->ev_tgt_in) HIPTRY(hipEventCreateWithFlags(&ctx->ev_tgt_in, hipEventDisableTiming));
    if (!ctx->copy_tgt) HIPTRY(hipStreamCreateWithFlags(&ctx->copy_tgt, hipStreamNonBlocking));
    if (!ctx->copy_ref) HIPTRY(hipStreamCreateWithFlags(&ctx->copy_ref, hipStreamNonBlocking));
    return 0;
}

// whole contents of an open descriptor that is not a regular file (a FIFO, /dev/stdin, a process
// substitution): read to EOF, as the reference's ifstream + getline loop does (compression.cpp:186-218)
bool slurp_fd(int fd, std::vector<uint8_t>* v) {
    v->clear();
    size_t n = 0;
    for (;;) {
        if (v->size() - n < ((size_t)1 << 20)) v->resize(n + ((size_t)4 << 20));
        const ssize_t r = read(fd, v->data() + n, v->size() - n);
        if (r < 0) {
            if (errno == EINTR) continue;
            return false;
        }
        if (r == 0) break;
        n += (size_t)r;
    }
    v->resize(n);
    return true;
}

struct FileLoad {
    sccg_ctx* ctx;
    int fd[2];                 // 0 reference, 1 target
    int64_t len[2];
    uint8_t* dst[2];           // device
    int64_t npiece[2];
    std::mutex mu;
    std::condition_variable cv;
    int64_t queued[2] = {0, 0};
    int err = 0;               // first failure: SCCG_E_OPEN_REF / SCCG_E_OPEN_TGT / SCCG_E_HIP
    std::string msg;

    void fail(int code, const std::string& m) {
        std::lock_guard<std::mutex> g(mu);
        if (!err) { err = code; msg = m; }
        cv.notify_all();
    }
    // reader t: pieces t, t + STAGE_THREADS, ... of the sequence (reference pieces, then target's)
    void reader(int t) {
        (void)hipSetDevice(ctx->device);
        const int64_t total = npiece[0] + npiece[1];
        int k = 0;
        for (int64_t p = t; p < total; p += STAGE_THREADS) {
            { std::lock_guard<std::mutex> g(mu); if (err) return; }
            const int f = p < npiece[0] ? 0 : 1;
            const int64_t q = f ? p - npiece[0] : p;
            const int64_t off = q * (int64_t)STAGE_PIECE;
            const size_t n = (size_t)(len[f] - off < (int64_t)STAGE_PIECE ? len[f] - off : (int64_t)STAGE_PIECE);
            const int si = t * STAGE_SLOTS + (k++ % STAGE_SLOTS);
            if (hipEventSynchronize(ctx->stage_ev[si]) != hipSuccess) { fail(SCCG_E_HIP, "staging event"); return; }
            size_t got = 0;
            while (got < n) {
                const ssize_t r = pread(fd[f], ctx->stage[si] + got, n - got, (off_t)(off + (int64_t)got));
                if (r <= 0) {
                    if (r < 0 && errno == EINTR) continue;
                    fail(f ? SCCG_E_OPEN_TGT : SCCG_E_OPEN_REF, f ? "short read of the target file" : "short read of the reference file");
                    return;
                }
                got += (size_t)r;
            }
            hipStream_t cs = f ? ctx->copy_tgt : ctx->copy_ref;
            std::lock_guard<std::mutex> g(mu);   // the count and the copy's place on the stream together
            if (hipMemcpyAsync(dst[f] + off, ctx->stage[si], n, hipMemcpyHostToDevice, cs) != hipSuccess ||
                hipEventRecord(ctx->stage_ev[si], cs) != hipSuccess) {
                if (!err) { err = SCCG_E_HIP; msg = "staging copy"; }
                cv.notify_all();
                return;
            }
            queued[f]++;
            cv.notify_all();
        }
    }
    // blocks until every piece of file f is queued; records ev behind them on f's copy stream
    int ready(int f, hipEvent_t ev) {
        std::unique_lock<std::mutex> lk(mu);
        cv.wait(lk, [&] { return err || queued[f] == npiece[f]; });
        if (err) return err;
        if (hipEventRecord(ev, f ? ctx->copy_tgt : ctx->copy_ref) != hipSuccess) return SCCG_E_HIP;
        return 0;
    }
    static int ref_ready(void* u, hipEvent_t* e) {
        FileLoad* L = static_cast<FileLoad*>(u);
        *e = L->ctx->ev_ref_in;
        return L->ready(0, *e);
    }
    static int tgt_ready(void* u, hipEvent_t* e) {
        FileLoad* L = static_cast<FileLoad*>(u);
        *e = L->ctx->ev_tgt_in;
        return L->ready(1, *e);
    }
};

int write_all(int fd, const uint8_t* p, size_t n) {
    while (n) {
        const ssize_t w = write(fd, p, n);
        if (w < 0) {
            if (errno == EINTR) continue;
            return -1;
        }
        p += w;
        n -= (size_t)w;
    }
    return 0;
}

int compress_files_impl(sccg_ctx* ctx, const sccg_params& P, const char* ref_path, const char* tgt_path,
                        const char* out_path, int64_t* out_len) {
    // open both inputs first, in the reference's order and with its failure points (:187-191, :202-206)
    struct Fd {
        int v = -1;
        ~Fd() { if (v >= 0) close(v); }
    } fr, ft;
    fr.v = open(ref_path, O_RDONLY);
    if (fr.v < 0) return ctx->fail(SCCG_E_OPEN_REF, "Error opening reference file: %s", ref_path);
    ft.v = open(tgt_path, O_RDONLY);
    if (ft.v < 0) return ctx->fail(SCCG_E_OPEN_TGT, "Error opening target file: %s", tgt_path);
    struct stat sr{}, stt{};
    const bool reg_r = !fstat(fr.v, &sr) && S_ISREG(sr.st_mode);
    const bool reg_t = !fstat(ft.v, &stt) && S_ISREG(stt.st_mode);
    if (!reg_r || !reg_t) {
        // a FIFO / pipe / character device has no size to stage by: read both to EOF into host
        // memory (reference first, as the reference does) and take the host path
        std::vector<uint8_t> hr, ht;
        if (!slurp_fd(fr.v, &hr)) return ctx->fail(SCCG_E_OPEN_REF, "Error reading reference file: %s", ref_path);
        if (!slurp_fd(ft.v, &ht)) return ctx->fail(SCCG_E_OPEN_TGT, "Error reading target file: %s", tgt_path);
        sccg_buf b{nullptr, 0};
        const int rc = sccg_compress_ex(ctx, &P, (const char*)hr.data(), hr.size(), (const char*)ht.data(), ht.size(), &b);
        if (rc && rc != SCCG_E_DELTA_STOI) { sccg_buf_free(&b); return rc; }
        Fd fo;
        fo.v = open(out_path, O_WRONLY | O_CREAT | O_TRUNC, 0644);
        const bool ok = fo.v >= 0 && !write_all(fo.v, (const uint8_t*)b.data, b.len);
        const int64_t n = (int64_t)b.len;
        sccg_buf_free(&b);
        if (!ok) return ctx->fail(SCCG_E_WRITE, "cannot write %s", out_path);
        if (close(fo.v)) { fo.v = -1; return ctx->fail(SCCG_E_WRITE, "closing %s failed", out_path); }
        fo.v = -1;
        *out_len = n;
        return rc;
    }
    TRY(staging_init(ctx));
    const int64_t rn = (int64_t)sr.st_size, tn = (int64_t)stt.st_size;
    uint8_t* drf = reinterpret_cast<uint8_t*>(ctx->get(B_RFA, (size_t)rn + 16));
    uint8_t* dtf = reinterpret_cast<uint8_t*>(ctx->get(B_TFA, (size_t)tn + 16));
    const size_t cap = sccg_compress_bound((size_t)rn, (size_t)tn);
    uint8_t* dout = reinterpret_cast<uint8_t*>(ctx->get(B_OUT, cap));
    if (!drf || !dtf || !dout) return ctx->fail(SCCG_E_NOMEM, "device allocation failed");

    FileLoad L;
    L.ctx = ctx;
    L.fd[0] = fr.v; L.fd[1] = ft.v;
    L.len[0] = rn; L.len[1] = tn;
    L.dst[0] = drf; L.dst[1] = dtf;
    L.npiece[0] = (rn + (int64_t)STAGE_PIECE - 1) / (int64_t)STAGE_PIECE;
    L.npiece[1] = (tn + (int64_t)STAGE_PIECE - 1) / (int64_t)STAGE_PIECE;
    std::vector<std::thread> th;
    for (int t = 0; t < STAGE_THREADS; t++) th.emplace_back([&L, t] { L.reader(t); });
    struct Join {   // every exit path: the readers joined, then their queued copies drained (a later
        std::vector<std::thread>& th;   // ctx->get() may reallocate the buffers they write into)
        sccg_ctx* ctx;
        ~Join() {
            for (auto& x : th) if (x.joinable()) x.join();
            (void)hipStreamSynchronize(ctx->copy_ref);
            (void)hipStreamSynchronize(ctx->copy_tgt);
        }
    } join{th, ctx};
    const InputReady rdy{&FileLoad::ref_ready, &FileLoad::tgt_ready, &L};
    int64_t len = 0;
    int rc = compress_device_impl(ctx, P, drf, rn, dtf, tn, dout, (int64_t)cap, &len, &rdy);
    for (auto& x : th) x.join();
    if (L.err) return ctx->fail(L.err, "%s", L.msg.c_str());
    if (rc && rc != SCCG_E_DELTA_STOI) return rc;   // DELTA_STOI still writes the file's text
    // the record file (compression.cpp:329-331): a piece at a time through the pinned slots
    Fd fo;
    fo.v = open(out_path, O_WRONLY | O_CREAT | O_TRUNC, 0644);
    if (fo.v < 0) return ctx->fail(SCCG_E_WRITE, "cannot open %s for writing", out_path);
    const int64_t np = (len + (int64_t)STAGE_PIECE - 1) / (int64_t)STAGE_PIECE;
    for (int64_t p = 0; p < np + 1; p++) {
        if (p < np) {   // copy piece p while piece p - 1 is written
            const int64_t off = p * (int64_t)STAGE_PIECE;
            const size_t n = (size_t)(len - off < (int64_t)STAGE_PIECE ? len - off : (int64_t)STAGE_PIECE);
            HIPTRY(hipMemcpyAsync(ctx->stage[p & 1], dout + off, n, hipMemcpyDeviceToHost, ctx->stream));
            HIPTRY(hipEventRecord(ctx->stage_ev[p & 1], ctx->stream));
        }
        if (p > 0) {
            const int64_t q = p - 1, off = q * (int64_t)STAGE_PIECE;
            const size_t n = (size_t)(len - off < (int64_t)STAGE_PIECE ? len - off : (int64_t)STAGE_PIECE);
            HIPTRY(hipEventSynchronize(ctx->stage_ev[q & 1]));
            if (write_all(fo.v, ctx->stage[q & 1], n)) return ctx->fail(SCCG_E_WRITE, "write to %s failed", out_path);
        }
    }
    if (close(fo.v)) { fo.v = -1; return ctx->fail(SCCG_E_WRITE, "closing %s failed", out_path); }
    fo.v = -1;
    *out_len = len;
    return rc;
}

// -------------------------------------------------------------------------------------------
// reconstruction (decompression.cpp)
// -------------------------------------------------------------------------------------------
int reconstruct_impl(sccg_ctx* ctx, const uint8_t* rfa, int64_t rn, const uint8_t* rec, int64_t n, uint8_t* out,
                     int64_t out_cap, int64_t* out_len, bool size_only) {
    hipStream_t s = ctx->stream;
    GET(int64_t, sc, B_SCAL, 64);
    // ---- reference (decompression.cpp:47-58, 105-110), first, on the side stream beside everything
    //      that follows: its filter depends on the N line only when that line is exactly "," (then it
    //      keeps the N's, FILTER_UPPER), so the usual filter starts now and that rare case redoes it
    //      once the lines are known.  (Its length |R'| stays on the device, sc[9], until the range
    //      check and the parse's readback.)
    GET(uint8_t, Rp, B_RP, rn + 64);   // (only R' is read: the strip writes no R here)
    HIPTRY(hipEventRecord(ctx->ev_fork, s));
    HIPTRY(hipStreamWaitEvent(ctx->side, ctx->ev_fork, 0));
    TRY(strip(ctx, INGEST_REF, rfa, rn, nullptr, nullptr, sc + 8, nullptr, nullptr, FILTER_DROP_UPPERN_ONLY, Rp, 1, ctx->side));
    HIPTRY(hipEventRecord(ctx->ev_rstrip, ctx->side));
    struct JoinSide {   // every exit path: the main stream waits for the strip (a later call reuses Rp)
        sccg_ctx* c;
        hipStream_t st;
        ~JoinSide() { (void)hipStreamWaitEvent(st, c->ev_rstrip, 0); }
    } join_side{ctx, s};
    // the line ends: one pass collects every '\n' (a record file holds 2-3); more than DC_NL_CAP
    // of them -> four ordered first-match searches.  (Queued ahead of the strip, the search itself
    // finished earlier, but its one-wave readback then waited ~40 us for a slot behind the strip's
    // grid: measured slower.)
    int64_t nl[4];
    int64_t nlb[1 + DC_NL_CAP];
    uint8_t first = 0;
    GET(int64_t, dnl, B_D_NLPOS, 1 + DC_NL_CAP);
    int32_t* d_err = reinterpret_cast<int32_t*>(sc + 40);
    TRY(dc_newlines(rec, n, dnl, s, d_err));   // (also zeroes the error bits)
    {
        const RbItem it[2] = {{dnl, nlb, (int)sizeof nlb}, {rec, &first, n > 0 ? 1 : 0}};
        TRY(dev_readback(it, 2, s));
    }
    if (nlb[0] <= DC_NL_CAP) {
        std::sort(nlb + 1, nlb + 1 + nlb[0]);
        for (int i = 0; i < 4; i++) nl[i] = i < nlb[0] ? nlb[1 + i] : n;
    } else {
        TRY(dc_find_lines(rec, n, sc, s));
        const RbItem it{sc, nl, (int)sizeof nl};
        TRY(dev_readback(&it, 1, s));
    }
    // getline semantics: line i spans [start_i, nl_i); it exists iff start_i < n  (:68-97)
    int64_t start[4], end[4];
    start[0] = 0;
    for (int i = 0; i < 4; i++) {
        end[i] = nl[i];
        if (i < 3) start[i + 1] = nl[i] + 1;
    }
    if (n <= 0) return ctx->fail(SCCG_E_FORMAT, "empty record file");
    const bool has_hdr = end[0] > 0 && first == '>';
    const int li = has_hdr ? 1 : 0;
    for (int i = 1; i <= li + 2; i++)
        if (start[i] >= n + (i == 0)) return ctx->fail(SCCG_E_FORMAT, "record file misses line %d", i + 1);
    const uint8_t* lower = rec + start[li];
    const int64_t nlower = end[li] - start[li];
    const uint8_t* nline = rec + start[li + 1];
    const int64_t nnl = end[li + 1] - start[li + 1];
    const uint8_t* enc = rec + start[li + 2];
    const int64_t nenc = end[li + 2] - start[li + 2];

    bool n_is_comma = false;
    if (nnl == 1) {
        uint8_t c = 0;
        const RbItem it{nline, &c, 1};
        TRY(dev_readback(&it, 1, s));
        n_is_comma = c == ',';
    }
    if (n_is_comma) {   // the N line is ",": the reference keeps its N's (redo the strip behind the first)
        HIPTRY(hipEventRecord(ctx->ev_fork, s));
        HIPTRY(hipStreamWaitEvent(ctx->side, ctx->ev_fork, 0));
        TRY(strip(ctx, INGEST_REF, rfa, rn, nullptr, nullptr, sc + 8, nullptr, nullptr, FILTER_UPPER, Rp, 1, ctx->side));
        HIPTRY(hipEventRecord(ctx->ev_rstrip, ctx->side));
    }

    // ---- record line on side2 (own scratch) beside the run-line parses, which read counts back
    GET(int64_t, lp2, B_D_LP2, nenc + 1);
    GET(int64_t, dlt2, B_D_DLT2, nenc + 1);
    GET(int64_t, part2, B_PARTIAL2, scan_partials_needed(nenc + 1) + 16);
    GET(int64_t, contrib, B_D_CONTRIB, nenc + 1);
    GET(int64_t, doff, B_D_OFF, nenc + 1);
    GET(int64_t, dsum, B_D_DSUM, nenc + 1);
    const int64_t nmax = nlower > nnl ? nlower : nnl;   // >= dc_run_cap of either line but for n <= 3
    GET(int64_t, lp, B_D_LP, nmax + 4);
    // (the tiled run-line parser keeps 4 + 256 int64 per 1 KiB tile in flag / dlt: <= n / 4 + 260)
    GET(int64_t, flag, B_D_FLAG, nmax + 4 + 264);
    GET(int64_t, dlt, B_D_DLT, nmax + 4 + 264);
    GET(int64_t, part, B_PARTIAL, scan_partials_needed(nmax + 4) + 16);
    GET(int32_t, ls, B_D_LS, dc_run_cap(nlower));
    GET(int32_t, ll, B_D_LL, dc_run_cap(nlower));
    GET(int64_t, lc, B_D_LC, dc_run_cap(nlower));
    GET(int32_t, ns, B_D_NS, dc_run_cap(nnl));
    GET(int32_t, nlr, B_D_NL, dc_run_cap(nnl));
    GET(int64_t, nc, B_D_NC, dc_run_cap(nnl));
    // fused path: the record line becomes a token table (no R' needed) that the formatter expands
    const bool fused = dc_fused() && rn < ((int64_t)1 << 31) && nenc < ((int64_t)1 << 31);   // (32-bit sources)
    DcTokBuf tk{};
    const int64_t tcap = dc_tok_cap(nenc > 0 ? nenc : 0);
    if (fused) {
        GET(int64_t, tkb, B_D_TOK, 4 * tcap);
        tk.tab = DcTokTab{tkb, tkb + tcap, tkb + 2 * tcap, tkb + 3 * tcap};
        const int64_t nbk = (nenc > 0 ? nenc : 0) / 64 + 2;
        GET(int64_t, btk, B_D_BTOK, 2 * nbk);
        tk.btok = btk;
        tk.btoff = btk + nbk;
        tk.d_ntok = sc + 24;
    }
    HIPTRY(hipEventRecord(ctx->ev_fork2, s));
    HIPTRY(hipStreamWaitEvent(ctx->side2, ctx->ev_fork2, 0));
    // The host issues launches one at a time, so the chain issued first starts ~40 us earlier.
    // Round 6: the run lines' chain (side2) is the critical one -- with the reference strip's
    // write pass shortened, the record line's token blocks end ~70 us before the run lines'
    // parse on chr1 (profiles/r06/dprof_timeline.txt) -- so it goes first (SCCG_DC_RUNS_FIRST=0:
    // the record line's chain first, as in round 5, when the strip's grid delayed the token blocks).
    // The two are joined before the N check.
    static const bool runs_first = [] { const char* e = getenv("SCCG_DC_RUNS_FIRST"); return !e || atoi(e) > 0; }();
    DcRuns lr{}, nr{};
    lr.start = ls; lr.len = ll; lr.cum = lc;
    nr.start = ns; nr.len = nlr; nr.cum = nc;
    if (runs_first) {
        TRY(dc_parse_runs2(lower, nlower, &lr, sc + 14, nline, nnl, &nr, sc + 16, lp, flag, dlt, part, d_err, ctx->side2));
        HIPTRY(hipEventRecord(ctx->ev_lines, ctx->side2));
    }
    TRY(dc_decode_prepare(enc, nenc, lp2, contrib, dlt2, doff, dsum, sc + 9, ctx->ev_rstrip, part2, d_err, sc + 12,
                          s, fused ? &tk : nullptr));
    if (!runs_first) {
        TRY(dc_parse_runs2(lower, nlower, &lr, sc + 14, nline, nnl, &nr, sc + 16, lp, flag, dlt, part, d_err, ctx->side2));
        HIPTRY(hipEventRecord(ctx->ev_lines, ctx->side2));
    }
    HIPTRY(hipStreamWaitEvent(s, ctx->ev_lines, 0));
    // The usual call queues the token fill right behind the N check, before the host knows the
    // decoded length D, into a buffer of the output's capacity (D <= nres < out_cap whenever the
    // call succeeds; the fill writes nothing past it), and reads the lengths back on side2 beside
    // it: the fill no longer waits for a host round trip.  (SCCG_DC_SPEC=0: the fill after the
    // readback.  Queued behind the readback copy on the same stream it gained nothing: the copy,
    // an event and a cross-stream wait still sat between the N check and the fill.)
    constexpr int64_t SPEC_FILL_MAX = (int64_t)4 << 30;
    static const bool spec_on = [] { const char* e = getenv("SCCG_DC_SPEC"); return !e || atoi(e) != 0; }();
    // The speculative buffer is sized by the caller's capacity, not by D: a caller passing a far
    // larger output buffer than the record can need (D rarely exceeds |R| + |rec|: every token
    // copies reference bytes, every literal is a record byte) takes the non-speculative path, which
    // sizes it by D; so does a call whose speculative allocation fails.
    bool spec_fill = spec_on && !fused && dc_tok_tiled() && !size_only && nenc > 0 && out_cap > 0 &&
                     out_cap <= SPEC_FILL_MAX && out_cap <= 2 * (rn + n) + ((int64_t)64 << 20);
    uint8_t* dec_spec = nullptr;
    if (spec_fill) {
        dec_spec = reinterpret_cast<uint8_t*>(ctx->get(B_D_DEC, (size_t)out_cap + 64));
        if (!dec_spec) spec_fill = false;
    }
    // (the strip's wait goes ahead of the N check, so nothing but the fork's event sits between the
    // check and the fill; the strip has long finished by then on genome-sized records)
    if (!dc_tok_tiled() || spec_fill) HIPTRY(hipStreamWaitEvent(s, ctx->ev_rstrip, 0));
    TRY(dc_n_check(nr, sc + 16, sc + 12, d_err, s));
    uint8_t* dec = nullptr;
    hipStream_t rbs = s;
    if (spec_fill) {
        dec = dec_spec;
        HIPTRY(hipEventRecord(ctx->ev_fork2, s));
        TRY(dc_decode_fill(enc, nenc, lp2, doff, dsum, dlt2, contrib, Rp, dec, s, sc + 9, d_err, out_cap));
        HIPTRY(hipStreamWaitEvent(ctx->side2, ctx->ev_fork2, 0));
        rbs = ctx->side2;
    }
    // one readback: decoded length, error bits, both run lines' counts and totals -- with the tiled
    // record line (range check in the fill) it does not wait for the reference's strip, whose |R'|
    // is read with the final error bits
    int64_t D = 0, nRp = 0, cnt[4] = {0, 0, 0, 0};
    int32_t err = 0;
    {
        const RbItem it[3] = {{sc + 12, &D, (int)sizeof D}, {d_err, &err, (int)sizeof err}, {sc + 14, cnt, (int)sizeof cnt}};
        TRY(dev_readback(it, 3, rbs));
    }
    lr.n = cnt[0]; lr.total = cnt[1];
    nr.n = cnt[2]; nr.total = cnt[3];
    if (err & 1) return ctx->fail(SCCG_E_PARSE, "record text outside the run/token grammar");
    if (err & 2) return ctx->fail(SCCG_E_RANGE, "token exceeds the reference (decompression.cpp:223-229)");
    const int64_t nres = D + nr.total;
    const int64_t hlen = has_hdr ? end[0] : 0;
    const int64_t total = hlen + 1 + nres + (nres > 0 ? (nres - 1) / 50 : 0) + 1;
    if (!fused && dc_tok_tiled() && (size_only || (err & 4) || total > out_cap)) {
        // the tiled record line checks the token range in its fill: a size query or an early error
        // runs that check alone first, so it reports SCCG_E_RANGE as the full decode (and the
        // reference, which exits at :223-229 before it places N) would
        HIPTRY(hipStreamWaitEvent(s, ctx->ev_rstrip, 0));
        TRY(dc_tok_range_tiled(enc, nenc, lp2, doff, dsum, sc + 9, d_err, s));
        const RbItem it{d_err, &err, (int)sizeof err};
        TRY(dev_readback(&it, 1, s));
        if (err & 2) return ctx->fail(SCCG_E_RANGE, "token exceeds the reference (decompression.cpp:223-229)");
    }
    if (err & 4) return ctx->fail(SCCG_E_PARSE, "N positions beyond the sequence");
    *out_len = total;
    if (size_only) return SCCG_OK;
    if (total > out_cap) return ctx->fail(SCCG_E_NOMEM, "output needs %lld bytes", (long long)total);
    if (fused) {
        // range check after the strip on side2; the formatter expands the tokens straight from R'
        HIPTRY(hipStreamWaitEvent(ctx->side2, ctx->ev_rstrip, 0));
        TRY(dc_tok_range(tk, tcap, sc + 9, d_err, ctx->side2));
        HIPTRY(hipEventRecord(ctx->ev_lines, ctx->side2));
        if (hlen) HIPTRY(hipMemcpyAsync(out, rec, (size_t)hlen, hipMemcpyDeviceToDevice, s));
        TRY(dev_put_bytes(out + hlen, "\n", 1, s));
        GET(int64_t, span, B_D_SPAN, dc_format_span_words(nres));
        const DcFmtSrc fz{tk.tab, tk.d_ntok, enc, nenc > 0 ? nenc : 0, Rp, sc + 9};
        TRY(dc_format(nullptr, nres, nr, lr, span, out + hlen + 1, s, &fz, ctx->ev_rstrip));
        TRY(dev_put_bytes(out + total - 1, "\n", 1, s));
        HIPTRY(hipStreamWaitEvent(s, ctx->ev_lines, 0));
        const RbItem it[2] = {{d_err, &err, (int)sizeof err}, {sc + 9, &nRp, (int)sizeof nRp}};
        TRY(dev_readback(it, 2, s));
        if (err & 2) return ctx->fail(SCCG_E_RANGE, "token exceeds the reference (decompression.cpp:223-229)");
        ctx->stats.target_bases = nres;
        ctx->stats.reference_bases = nRp;
        return SCCG_OK;
    }
    if (!spec_fill) {   // (the fill is launched first: it is the critical path)
        GET(uint8_t, dec1, B_D_DEC, D + 64);
        dec = dec1;
        HIPTRY(hipEventRecord(ctx->ev_fork2, s));
        HIPTRY(hipStreamWaitEvent(s, ctx->ev_rstrip, 0));   // the fill copies from R'
        TRY(dc_decode_fill(enc, nenc, lp2, doff, dsum, dlt2, contrib, Rp, dec, s, sc + 9, d_err));
        HIPTRY(hipStreamWaitEvent(ctx->side2, ctx->ev_fork2, 0));
    }
    GET(int64_t, span, B_D_SPAN, dc_format_span_words(nres));
    // side2, beside the token fill: the output's frame (header, its '\n', the final '\n' -- bytes
    // the formatter does not write) and the formatter's block index (run lists only)
    TRY(dev_put_frame(out, rec, hlen, total, ctx->side2));
    int irc = 0;
    const bool index_ready = dc_format_index(nres, nr, lr, span, out + hlen + 1, ctx->side2, &irc);
    TRY(irc);
    HIPTRY(hipEventRecord(ctx->ev_lines, ctx->side2));
    TRY(dc_format(dec, nres, nr, lr, span, out + hlen + 1, s, nullptr, ctx->ev_lines, index_ready));
    {   // (tiled record line: the range check ran with the fill) error bits and |R'| behind the output
        const RbItem it[2] = {{d_err, &err, (int)sizeof err}, {sc + 9, &nRp, (int)sizeof nRp}};
        TRY(dev_readback(it, 2, s));
        if (err & 2) return ctx->fail(SCCG_E_RANGE, "token exceeds the reference (decompression.cpp:223-229)");
    }
    ctx->stats.target_bases = nres;
    ctx->stats.reference_bases = nRp;
    return SCCG_OK;
}

}  // namespace

extern "C" {

void sccg_params_default(sccg_params* p) {
    if (!p) return;
    p->k = 14; p->k2 = 10; p->L = SEG_L; p->m = 100; p->T1 = 0.5f; p->T2 = 4; p->local = 1;   // compression.cpp:373-379
}

int sccg_compress_device_ex(sccg_ctx* ctx, const sccg_params* params, const void* d_ref_fa, size_t ref_len,
                            const void* d_tgt_fa, size_t tgt_len, void* d_out, size_t out_cap, size_t* out_len, void* stream) {
    if (!ctx || !params || !d_out || !out_len || (!d_ref_fa && ref_len) || (!d_tgt_fa && tgt_len)) return SCCG_E_INVALID;
    HIPTRY(hipSetDevice(ctx->device));
    hipStream_t saved = ctx->stream;
    if (stream) ctx->stream = (hipStream_t)stream;
    int64_t len = 0;
    int rc = compress_device_impl(ctx, *params, (const uint8_t*)d_ref_fa, (int64_t)ref_len, (const uint8_t*)d_tgt_fa,
                                  (int64_t)tgt_len, (uint8_t*)d_out, (int64_t)out_cap, &len);
    ctx->stream = saved;
    *out_len = (size_t)len;
    return rc;
}

int sccg_compress_device(sccg_ctx* ctx, const void* d_ref_fa, size_t ref_len, const void* d_tgt_fa, size_t tgt_len,
                         void* d_out, size_t out_cap, size_t* out_len, void* stream) {
    sccg_params p;
    sccg_params_default(&p);
    return sccg_compress_device_ex(ctx, &p, d_ref_fa, ref_len, d_tgt_fa, tgt_len, d_out, out_cap, out_len, stream);
}

int sccg_compress(sccg_ctx* ctx, const char* ref_fa, size_t ref_len, const char* tgt_fa, size_t tgt_len,
                  sccg_buf* out_text) {
    sccg_params p;
    sccg_params_default(&p);
    return sccg_compress_ex(ctx, &p, ref_fa, ref_len, tgt_fa, tgt_len, out_text);
}

int sccg_compress_ex(sccg_ctx* ctx, const sccg_params* params, const char* ref_fa, size_t ref_len, const char* tgt_fa,
                     size_t tgt_len, sccg_buf* out_text) {
    if (!ctx || !params || !out_text || (!ref_fa && ref_len) || (!tgt_fa && tgt_len)) return SCCG_E_INVALID;
    out_text->data = nullptr;
    out_text->len = 0;
    HIPTRY(hipSetDevice(ctx->device));
    uint8_t* drf = reinterpret_cast<uint8_t*>(ctx->get(B_RFA, ref_len + 16));
    uint8_t* dtf = reinterpret_cast<uint8_t*>(ctx->get(B_TFA, tgt_len + 16));
    const size_t cap = sccg_compress_bound(ref_len, tgt_len);
    uint8_t* dout = reinterpret_cast<uint8_t*>(ctx->get(B_OUT, cap));
    if (!drf || !dtf || !dout) return ctx->fail(SCCG_E_NOMEM, "device allocation failed");
    if (ref_len) HIPTRY(hipMemcpyAsync(drf, ref_fa, ref_len, hipMemcpyHostToDevice, ctx->stream));
    if (tgt_len) HIPTRY(hipMemcpyAsync(dtf, tgt_fa, tgt_len, hipMemcpyHostToDevice, ctx->stream));
    int64_t len = 0;
    int rc = compress_device_impl(ctx, *params, drf, (int64_t)ref_len, dtf, (int64_t)tgt_len, dout, (int64_t)cap, &len);
    if (rc && rc != SCCG_E_DELTA_STOI) return rc;   // DELTA_STOI still returns the file's text
    char* h = (char*)malloc((size_t)len + 1);
    if (!h) return ctx->fail(SCCG_E_NOMEM, "host allocation failed");
    if (len) HIPTRY(hipMemcpy(h, dout, (size_t)len, hipMemcpyDeviceToHost));
    h[len] = 0;
    out_text->data = h;
    out_text->len = (size_t)len;
    return rc;
}

int sccg_compress_files(sccg_ctx* ctx, const sccg_params* params, const char* ref_path, const char* tgt_path,
                        const char* out_path, size_t* out_len) {
    if (!ctx || !ref_path || !tgt_path || !out_path) return SCCG_E_INVALID;
    sccg_params p;
    sccg_params_default(&p);
    if (params) p = *params;
    HIPTRY(hipSetDevice(ctx->device));
    int64_t len = 0;
    const int rc = compress_files_impl(ctx, p, ref_path, tgt_path, out_path, &len);
    if (out_len) *out_len = (size_t)len;
    return rc;
}

int sccg_reconstruct_device(sccg_ctx* ctx, const void* d_ref_fa, size_t ref_len, const void* d_rec, size_t rec_len,
                            void* d_out, size_t out_cap, size_t* out_len, void* stream) {
    if (!ctx || !out_len || (!d_ref_fa && ref_len) || (!d_rec && rec_len)) return SCCG_E_INVALID;
    HIPTRY(hipSetDevice(ctx->device));
    hipStream_t saved = ctx->stream;
    if (stream) ctx->stream = (hipStream_t)stream;
    int64_t len = 0;
    int rc = reconstruct_impl(ctx, (const uint8_t*)d_ref_fa, (int64_t)ref_len, (const uint8_t*)d_rec, (int64_t)rec_len,
                              (uint8_t*)d_out, (int64_t)out_cap, &len, d_out == nullptr);
    ctx->stream = saved;
    *out_len = (size_t)len;
    return rc;
}

int sccg_reconstruct(sccg_ctx* ctx, const char* ref_fa, size_t ref_len, const char* rec_text, size_t rec_len,
                     sccg_buf* out_fa) {
    if (!ctx || !out_fa || (!ref_fa && ref_len) || (!rec_text && rec_len)) return SCCG_E_INVALID;
    out_fa->data = nullptr;
    out_fa->len = 0;
    HIPTRY(hipSetDevice(ctx->device));
    uint8_t* drf = reinterpret_cast<uint8_t*>(ctx->get(B_RFA, ref_len + 16));
    uint8_t* drc = reinterpret_cast<uint8_t*>(ctx->get(B_TFA, rec_len + 16));
    if (!drf || !drc) return ctx->fail(SCCG_E_NOMEM, "device allocation failed");
    if (ref_len) HIPTRY(hipMemcpyAsync(drf, ref_fa, ref_len, hipMemcpyHostToDevice, ctx->stream));
    if (rec_len) HIPTRY(hipMemcpyAsync(drc, rec_text, rec_len, hipMemcpyHostToDevice, ctx->stream));
    int64_t need = 0;
    int rc = reconstruct_impl(ctx, drf, (int64_t)ref_len, drc, (int64_t)rec_len, nullptr, 0, &need, true);
    if (rc) return rc;
    uint8_t* dout = reinterpret_cast<uint8_t*>(ctx->get(B_OUT, (size_t)need + 16));
    if (!dout) return ctx->fail(SCCG_E_NOMEM, "device allocation failed");
    int64_t len = 0;
    rc = reconstruct_impl(ctx, drf, (int64_t)ref_len, drc, (int64_t)rec_len, dout, need + 16, &len, false);
    if (rc) return rc;
    char* h = (char*)malloc((size_t)len + 1);
    if (!h) return ctx->fail(SCCG_E_NOMEM, "host allocation failed");
    HIPTRY(hipMemcpy(h, dout, (size_t)len, hipMemcpyDeviceToHost));
    h[len] = 0;
    out_fa->data = h;
    out_fa->len = (size_t)len;
    return SCCG_OK;
}

// match_sequences seam (compression.cpp:36): local segments or the windowed global walk
// the walk from a state over device-resident R', T' (one chromosome's walk split
// across ranks, multigpu.split_walk): matches as kind-1 records with their target index
int walk_range_dev(sccg_ctx* ctx, const uint8_t* R, int64_t nr, const uint8_t* T, int64_t nt, int k, int m, int64_t x0,
                   int64_t P0, int64_t x_end, sccg_records* out, int64_t* exit_state, hipStream_t s) {
    if (m < 0 || 2 * m + 1 > 256 || k < 1 || k > 32 || nr >= (int64_t)INT32_MAX - 8 || nt >= (int64_t)INT32_MAX - 8)
        return ctx->fail(SCCG_E_UNSUPPORTED, "sccg_walk_range takes 0 <= m <= 127, 1 <= k <= 32");
    if (x0 < 0 || x0 > nt || P0 < -1 || P0 >= (nr > 0 ? nr : 1) || (P0 == -1 && x0 != 0))
        return ctx->fail(SCCG_E_UNSUPPORTED, "sccg_walk_range: state (x0, P0) outside the walk's states");
    const size_t wsb = walk_workspace_bytes(nr, nt, k, walk_chunk(nt));
    void* ws = ctx->get(B_WALK, wsb);
    if (!ws) return ctx->fail(SCCG_E_NOMEM, "walk workspace");
    WalkResult wr{};
    int64_t ex = 0, ep = -1;
    TRY(global_walk_range(R, nr, T, nt, k, m, walk_chunk(nt), ws, wsb, x0, P0, x_end, &ex, &ep, &wr, s));
    const int32_t *dt, *dp, *dl;
    int64_t nm;
    global_matches(ws, &dt, &dp, &dl, &nm);
    const size_t n = (size_t)nm;
    out->n = nm;
    out->kind = (uint8_t*)malloc(n ? n : 1);
    out->pos = (int32_t*)malloc((n ? n : 1) * 4);
    out->len = (int32_t*)malloc((n ? n : 1) * 4);
    out->t = (int64_t*)malloc((n ? n : 1) * 8);
    std::vector<int32_t> ht(n ? n : 1);
    const int rc = [&]() -> int {   // every error after the allocations frees them
        if (!out->kind || !out->pos || !out->len || !out->t) return ctx->fail(SCCG_E_NOMEM, "host allocation");
        if (n) {
            HIPTRY(hipMemcpyAsync(ht.data(), dt, n * 4, hipMemcpyDeviceToHost, s));
            HIPTRY(hipMemcpyAsync(out->pos, dp, n * 4, hipMemcpyDeviceToHost, s));
            HIPTRY(hipMemcpyAsync(out->len, dl, n * 4, hipMemcpyDeviceToHost, s));
        }
        HIPTRY(hipStreamSynchronize(s));
        return SCCG_OK;
    }();
    if (rc) {
        sccg_records_free(out);
        return rc;
    }
    for (size_t i = 0; i < n; i++) { out->kind[i] = 1; out->t[i] = ht[i]; }
    exit_state[0] = ex;
    exit_state[1] = ep;
    ctx->stats = sccg_stats{};
    ctx->stats.mode_global = 1;
    ctx->stats.n_matches = nm;
    ctx->stats.walk_rounds = wr.rounds;
    ctx->stats.walk_chunks = wr.chunks;
    ctx->stats.target_bases = nt;
    ctx->stats.walk_reference_bases = nr;
    return SCCG_OK;
}

int sccg_walk_range_device(sccg_ctx* ctx, const void* d_ref, size_t nr, const void* d_tgt, size_t nt, int k, int m,
                           int64_t x0, int64_t P0, int64_t x_end, sccg_records* out, int64_t* exit_state, void* stream) {
    if (!ctx || !out || !exit_state || (!d_ref && nr) || (!d_tgt && nt)) return SCCG_E_INVALID;
    memset(out, 0, sizeof *out);
    HIPTRY(hipSetDevice(ctx->device));
    global_prepare_reset();   // buffers shared with compress: never reuse its preparation
    hipStream_t s = stream ? (hipStream_t)stream : ctx->stream;
    // the walk reads up to 4 KiB past both sequences (whole-wave compares, prefetches): it runs on
    // context copies with that slack, not on the caller's buffers
    GET(uint8_t, R, B_RP, nr + 64);
    GET(uint8_t, T, B_TP, nt + 64);
    if (nr) HIPTRY(hipMemcpyAsync(R, d_ref, nr, hipMemcpyDeviceToDevice, s));
    if (nt) HIPTRY(hipMemcpyAsync(T, d_tgt, nt, hipMemcpyDeviceToDevice, s));
    return walk_range_dev(ctx, R, (int64_t)nr, T, (int64_t)nt, k, m, x0, P0, x_end, out, exit_state, s);
}

int sccg_walk_range(sccg_ctx* ctx, const uint8_t* sr, size_t nr, const uint8_t* st, size_t nt, int k, int m, int64_t x0,
                    int64_t P0, int64_t x_end, sccg_records* out, int64_t* exit_state) {
    if (!ctx || !out || !exit_state || (!sr && nr) || (!st && nt)) return SCCG_E_INVALID;
    memset(out, 0, sizeof *out);
    HIPTRY(hipSetDevice(ctx->device));
    global_prepare_reset();
    hipStream_t s = ctx->stream;
    GET(uint8_t, R, B_RP, nr + 64);
    GET(uint8_t, T, B_TP, nt + 64);
    if (nr) HIPTRY(hipMemcpyAsync(R, sr, nr, hipMemcpyHostToDevice, s));
    if (nt) HIPTRY(hipMemcpyAsync(T, st, nt, hipMemcpyHostToDevice, s));
    return walk_range_dev(ctx, R, (int64_t)nr, T, (int64_t)nt, k, m, x0, P0, x_end, out, exit_state, s);
}

int sccg_match(sccg_ctx* ctx, const uint8_t* sr, size_t nr, const uint8_t* st, size_t nt, int k, int m, int global,
               int64_t offset, sccg_records* out) {
    if (!ctx || !out || (!sr && nr) || (!st && nt)) return SCCG_E_INVALID;
    memset(out, 0, sizeof *out);
    HIPTRY(hipSetDevice(ctx->device));
    hipStream_t s = ctx->stream;
    std::vector<uint8_t> kind;
    std::vector<int32_t> pos, len;
    std::vector<int64_t> tt;
    auto push = [&](uint8_t kd, int32_t p, int32_t l, int64_t t) {
        kind.push_back(kd); pos.push_back(p); len.push_back(l); tt.push_back(t);
    };
    if (!global) {
        if (nr > (size_t)SEG_L || nt > (size_t)SEG_L || (k != 14 && k != 10))
            return ctx->fail(SCCG_E_UNSUPPORTED, "local sccg_match takes |Sr|,|St| <= 1000 and k in {10,14}");
        GET(uint8_t, R, B_R, nr + 64);
        GET(uint8_t, T, B_T, nt + 64);
        GET(uint32_t, recs, B_RECS, SEG_REC_CAP);
        GET(SegStat, stat, B_STAT, 1);
        if (nr) HIPTRY(hipMemcpyAsync(R, sr, nr, hipMemcpyHostToDevice, s));
        if (nt) HIPTRY(hipMemcpyAsync(T, st, nt, hipMemcpyHostToDevice, s));
        TRY(launch_local_pass(k, 1, 0, R, (int64_t)nr, T, (int64_t)nt, 0, 1, recs, stat, s));
        SegStat hs;
        uint32_t hr[SEG_REC_CAP];
        HIPTRY(hipMemcpyAsync(&hs, stat, sizeof hs, hipMemcpyDeviceToHost, s));
        HIPTRY(hipMemcpyAsync(hr, recs, sizeof hr, hipMemcpyDeviceToHost, s));
        HIPTRY(hipStreamSynchronize(s));
        for (int i = 0; i < hs.nrec; i++) {
            const uint32_t r = hr[i];
            if (r >> 31) push(1, (int32_t)((r >> 11) & 0xfffff) + (int32_t)offset, (int32_t)(r & 0x7ff), -1);
            else push(0, 0, (int32_t)(r & 0x7ff), (int64_t)(r >> 11));
        }
        // match records carry no t: recover it from the running position
        int64_t t = 0;
        for (size_t i = 0; i < kind.size(); i++) { if (kind[i]) tt[i] = t; t += len[i]; }
    } else {
        if (m < 0 || 2 * m + 1 > 256 || k < 1 || k > 32 || nr >= (size_t)INT32_MAX - 8 || nt >= (size_t)INT32_MAX - 8)
            return ctx->fail(SCCG_E_UNSUPPORTED, "global sccg_match takes 0 <= m <= 127, 1 <= k <= 32");
        global_prepare_reset();   // buffers shared with compress: never reuse its preparation
        GET(uint8_t, R, B_RP, nr + 64);
        GET(uint8_t, T, B_TP, nt + 64);
        if (nr) HIPTRY(hipMemcpyAsync(R, sr, nr, hipMemcpyHostToDevice, s));
        if (nt) HIPTRY(hipMemcpyAsync(T, st, nt, hipMemcpyHostToDevice, s));
        const size_t wsb = walk_workspace_bytes((int64_t)nr, (int64_t)nt, k, walk_chunk((int64_t)nt));
        void* ws = ctx->get(B_WALK, wsb);
        GET(uint8_t, txt, B_OUT, 4 * nt + 64);
        if (!ws) return ctx->fail(SCCG_E_NOMEM, "walk workspace");
        WalkResult wr{};
        int64_t tl = 0;
        TRY(global_match_and_emit(R, (int64_t)nr, T, (int64_t)nt, k, m, walk_chunk((int64_t)nt), ws, wsb, txt, &tl, &wr, s));
        const int32_t *dt, *dp, *dl;
        int64_t nm;
        global_matches(ws, &dt, &dp, &dl, &nm);
        std::vector<int32_t> ht((size_t)nm), hp((size_t)nm), hl((size_t)nm);
        if (nm) {
            HIPTRY(hipMemcpyAsync(ht.data(), dt, (size_t)nm * 4, hipMemcpyDeviceToHost, s));
            HIPTRY(hipMemcpyAsync(hp.data(), dp, (size_t)nm * 4, hipMemcpyDeviceToHost, s));
            HIPTRY(hipMemcpyAsync(hl.data(), dl, (size_t)nm * 4, hipMemcpyDeviceToHost, s));
        }
        HIPTRY(hipStreamSynchronize(s));
        int64_t prev_end = 0;
        for (int64_t i = 0; i < nm; i++) {
            if (ht[i] > prev_end) push(0, 0, (int32_t)(ht[i] - prev_end), prev_end);
            push(1, hp[i] + (int32_t)offset, hl[i], ht[i]);
            prev_end = ht[i] + hl[i];
        }
        if ((int64_t)nt > prev_end) push(0, 0, (int32_t)((int64_t)nt - prev_end), prev_end);
    }
    const size_t n = kind.size();
    out->n = (int64_t)n;
    out->kind = (uint8_t*)malloc(n ? n : 1);
    out->pos = (int32_t*)malloc((n ? n : 1) * 4);
    out->len = (int32_t*)malloc((n ? n : 1) * 4);
    out->t = (int64_t*)malloc((n ? n : 1) * 8);
    if (!out->kind || !out->pos || !out->len || !out->t) return ctx->fail(SCCG_E_NOMEM, "host allocation");
    if (n) {
        memcpy(out->kind, kind.data(), n);
        memcpy(out->pos, pos.data(), n * 4);
        memcpy(out->len, len.data(), n * 4);
        memcpy(out->t, tt.data(), n * 8);
    }
    return SCCG_OK;
}

}  // extern "C"
