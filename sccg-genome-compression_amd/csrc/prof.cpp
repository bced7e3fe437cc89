// prof.cpp -- optional per-kernel HIP-event timing (sccg_profile / sccg_profile_get).
//
// When enabled, the launchers bracket their hot kernels with a pair of events recorded on the
// stream the kernel runs on, so the measured duration is that launch's device time and agrees
// with rocprofv3 --kernel-trace for the same kernel.  Disabled (the default) it costs one branch.
#include <hip/hip_runtime.h>

#include <cstring>
#include <mutex>
#include <string>
#include <vector>

#include "internal.h"

namespace {

struct Pending {
    int id;
    hipEvent_t a, b;
};

struct Registry {
    std::mutex mu;
    bool on = false;
    uint32_t mask = ~0u;   // families bracketed while on (bit = family index)
    std::vector<hipEvent_t> pool;
    std::vector<Pending> pending;
    double ms[PROF_COUNT] = {};
    int64_t n[PROF_COUNT] = {};
    uint64_t epoch = 0;   // bumped by sccg_profile: begin events of an earlier epoch are dropped

    hipEvent_t take() {
        if (!pool.empty()) {
            hipEvent_t e = pool.back();
            pool.pop_back();
            return e;
        }
        hipEvent_t e = nullptr;
        (void)hipEventCreate(&e);
        return e;
    }
    void drain() {   // fold completed pairs into the totals
        for (auto& p : pending) {
            (void)hipEventSynchronize(p.b);
            float t = 0.f;
            if (hipEventElapsedTime(&t, p.a, p.b) == hipSuccess) {
                ms[p.id] += t;
                n[p.id] += 1;
            }
            pool.push_back(p.a);
            pool.push_back(p.b);
        }
        pending.clear();
    }
};

Registry& reg() {
    static Registry r;
    return r;
}

const char* const NAMES[PROF_COUNT] = {
    "fasta_strip", "run_extract", "run_text", "local_segments", "local_pass_k10", "local_emit", "n_filter",
    "first_sweep_anchors", "walk", "presence_scan", "fullc_scan", "match_emit", "walk_chain",
    "dc_decode", "dc_format", "walk_carry",
};

// each host thread brackets its own launches (several contexts may launch the same family at once)
struct Open {
    hipEvent_t e[PROF_COUNT] = {};
    uint64_t epoch[PROF_COUNT] = {};
};
thread_local Open t_open;

}  // namespace

void prof_begin(hipStream_t s, int id) {
    Registry& r = reg();
    if (!r.on || !((r.mask >> id) & 1u)) return;
    std::lock_guard<std::mutex> g(r.mu);
    hipEvent_t e = r.take();
    (void)hipEventRecord(e, s);
    t_open.e[id] = e;
    t_open.epoch[id] = r.epoch;
}

void prof_end(hipStream_t s, int id) {
    Registry& r = reg();
    if (!r.on || !((r.mask >> id) & 1u)) return;
    std::lock_guard<std::mutex> g(r.mu);
    if (!t_open.e[id]) return;
    if (t_open.epoch[id] != r.epoch) { r.pool.push_back(t_open.e[id]); t_open.e[id] = nullptr; return; }
    hipEvent_t e = r.take();
    (void)hipEventRecord(e, s);
    r.pending.push_back({id, t_open.e[id], e});
    t_open.e[id] = nullptr;
    if (r.pending.size() > 4096) r.drain();
}

extern "C" {

int sccg_profile_mask(sccg_ctx* /*ctx*/, uint32_t mask) {
    Registry& r = reg();
    std::lock_guard<std::mutex> g(r.mu);
    r.drain();
    r.on = mask != 0;
    r.mask = mask;   // bit i: family sccg_profile_name(i)
    r.epoch++;
    for (int i = 0; i < PROF_COUNT; i++) { r.ms[i] = 0; r.n[i] = 0; }
    return SCCG_OK;
}

int sccg_profile(sccg_ctx* ctx, int enable) {
    return sccg_profile_mask(ctx, enable == 1 ? ~0u : (uint32_t)enable);
}

int sccg_profile_get(sccg_ctx* /*ctx*/, const char* kernel, double* total_ms, int64_t* launches) {
    if (!kernel || !total_ms || !launches) return SCCG_E_INVALID;
    Registry& r = reg();
    std::lock_guard<std::mutex> g(r.mu);
    r.drain();
    for (int i = 0; i < PROF_COUNT; i++) {
        if (!strcmp(NAMES[i], kernel)) {
            *total_ms = r.ms[i];
            *launches = r.n[i];
            return SCCG_OK;
        }
    }
    return SCCG_E_INVALID;
}

const char* sccg_profile_name(int i) { return (i >= 0 && i < PROF_COUNT) ? NAMES[i] : nullptr; }

}  // extern "C"
