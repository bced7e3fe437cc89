// delta.hip -- delta_encode (compression.cpp:222-304) as the reference runs it, for record lines
// whose literal bytes contain '('.
//
// The normal emitters write "(p - p_prev," directly, which equals delta_encode's output only when
// every '(' on the record line opens a real "(p,l)" token.  A literal '(' (a target byte) makes the
// reference's own token scan pair it with the next ')' -- usually the one closing the following
// real token -- and rewrite whatever stands before that token's first comma.  This file
// reproduces that scan exactly over the ABSOLUTE-position text the reference writes before
// delta_encode (compress_genome, compression.cpp:406-415/:564-573), data-parallel:
//
//   * the scan is a two-state automaton over the parenthesis bytes: after any '(' it is inside a
//     token, after any ')' outside.  So a '(' opens a token iff the last parenthesis before it is
//     a ')' (or there is none), a ')' closes one iff the last parenthesis before it is a '(' --
//     one max-scan ("last parenthesis strictly before i") decides both, and the k-th opener
//     pairs with the k-th closer (an opener without a closer ends the scan, :266-268);
//   * the token's first comma (:272) is the comma of rank (#commas before the opener);
//   * stoi (:279) is strtol on the text before that comma, failing when nothing converts or the
//     value leaves int; any failure makes the reference throw out of delta_encode before it
//     rewrites the file (it keeps the absolute text, main returns 1): SCCG_E_DELTA_STOI;
//   * delta = value - value of the previous comma token (0 first, :280-282, int wrap-around);
//     the text before the comma is replaced by to_string(delta) (:284-288);
//   * output offsets: an exclusive sum of per-token length changes, and per byte the last edit
//     at or before it (max-scan).
// Rare path (real genomes hold no '('): correctness over speed, but still all on the GPU.
#include "decomp.h"

namespace {

__global__ void k_dx_flags(const uint8_t* __restrict__ X, int64_t n, const int64_t* __restrict__ lp,
                           int64_t* __restrict__ fo, int64_t* __restrict__ fc, int64_t* __restrict__ fm) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        const uint8_t c = X[i];
        const int64_t l = lp[i];
        const uint8_t pc = l >= 0 ? X[l] : 0;
        fo[i] = c == '(' && pc != '(';
        fc[i] = c == ')' && pc == '(';
        fm[i] = c == ',';
    }
}

// ranks (exclusive sums of the flags) -> opener / closer / comma position lists
__global__ void k_dx_scatter(const uint8_t* __restrict__ X, int64_t n, const int64_t* __restrict__ lp,
                             const int64_t* __restrict__ ro, const int64_t* __restrict__ rc,
                             const int64_t* __restrict__ rm, int64_t* __restrict__ opos,
                             int64_t* __restrict__ cpos, int64_t* __restrict__ mpos) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        const uint8_t c = X[i];
        const int64_t l = lp[i];
        const uint8_t pc = l >= 0 ? X[l] : 0;
        if (c == '(' && pc != '(') opos[ro[i]] = i;
        if (c == ')' && pc == '(') cpos[rc[i]] = i;
        if (c == ',') mpos[rm[i]] = i;
    }
}

__device__ __forceinline__ bool c_isspace(uint8_t c) { return c == ' ' || (c >= '\t' && c <= '\r'); }

// strtol(base 10) over X[a, b) + stoi's int range check (compression.cpp:279)
__device__ bool stoi_like(const uint8_t* X, int64_t a, int64_t b, int32_t* v) {
    int64_t i = a;
    while (i < b && c_isspace(X[i])) i++;
    bool neg = false;
    if (i < b && (X[i] == '+' || X[i] == '-')) neg = X[i++] == '-';
    const int64_t d0 = i;
    uint64_t mag = 0;
    bool big = false;
    for (; i < b && X[i] >= '0' && X[i] <= '9'; i++) {
        mag = mag * 10 + (X[i] - '0');
        if (mag > (1ull << 31)) big = true, mag = 1ull << 32;   // saturate: out of int either way
    }
    if (i == d0) return false;                                   // invalid_argument
    if (big || mag > (neg ? (1ull << 31) : (1ull << 31) - 1)) return false;   // out_of_range
    *v = neg ? (int32_t)(0u - (uint32_t)mag) : (int32_t)mag;
    return true;
}

// per token: closer, first comma, value (sc: [0] openers, [1] closers, [2] commas, [4] error)
__global__ void k_dx_tokens(const uint8_t* __restrict__ X, const int64_t* __restrict__ rm,
                            const int64_t* __restrict__ opos, const int64_t* __restrict__ cpos,
                            const int64_t* __restrict__ mpos, int64_t* __restrict__ qpos,
                            int64_t* __restrict__ val, int64_t* __restrict__ hv, int64_t cap,
                            int64_t* __restrict__ sc) {
    const int64_t no = sc[0], nc = sc[1], nm = sc[2];
    for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < cap; t += (int64_t)gridDim.x * blockDim.x) {
        int64_t q = -1;
        if (t < no && t < nc) {
            const int64_t o = opos[t], c = cpos[t];
            const int64_t k = rm[o];
            if (k < nm && mpos[k] < c) q = mpos[k];
            if (q >= 0) {
                int32_t v = 0;
                if (!stoi_like(X, o + 1, q, &v)) atomicOr((unsigned long long*)&sc[4], 1ull);
                val[t] = v;
            }
        }
        qpos[t] = q;
        hv[t] = q >= 0 ? t : -1;
    }
}

// per comma token: delta against the previous comma token and the length change of its edit
__global__ void k_dx_shift(const int64_t* __restrict__ opos, const int64_t* __restrict__ qpos,
                           const int64_t* __restrict__ val, const int64_t* __restrict__ prevt,
                           int64_t* __restrict__ dl, int64_t* __restrict__ sh, int64_t cap) {
    for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < cap; t += (int64_t)gridDim.x * blockDim.x) {
        const int64_t q = qpos[t];
        if (q < 0) { sh[t] = 0; continue; }
        const int64_t pt = prevt[t];
        const int32_t prev = pt >= 0 ? (int32_t)val[pt] : 0;
        const int32_t d = (int32_t)((uint32_t)(int32_t)val[t] - (uint32_t)prev);
        dl[t] = d;
        sh[t] = ndigits_i32(d) - (q - opos[t] - 1);
    }
}

__global__ void k_dx_fill(int64_t* __restrict__ p, int64_t n, int64_t v) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
        p[i] = v;
}

__global__ void k_dx_mark(const int64_t* __restrict__ opos, const int64_t* __restrict__ qpos,
                          int64_t* __restrict__ E, int64_t cap) {
    for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < cap; t += (int64_t)gridDim.x * blockDim.x)
        if (qpos[t] >= 0) E[opos[t] + 1] = t;
}

// every byte not inside an edited prefix moves by the length changes of the edits before it
__global__ void k_dx_copy(const uint8_t* __restrict__ X, int64_t n, const int64_t* __restrict__ E,
                          const int64_t* __restrict__ Ex, const int64_t* __restrict__ qpos,
                          const int64_t* __restrict__ cs, const int64_t* __restrict__ sh,
                          uint8_t* __restrict__ out) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        const int64_t t = E[i] > Ex[i] ? E[i] : Ex[i];
        if (t < 0) { out[i] = X[i]; continue; }
        if (i < qpos[t]) continue;   // replaced text (o_t + 1 <= i < q_t)
        out[i + cs[t] + sh[t]] = X[i];
    }
}

__global__ void k_dx_edit(const int64_t* __restrict__ opos, const int64_t* __restrict__ qpos,
                          const int64_t* __restrict__ cs, const int64_t* __restrict__ dl,
                          uint8_t* __restrict__ out, int64_t cap) {
    for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < cap; t += (int64_t)gridDim.x * blockDim.x)
        if (qpos[t] >= 0) write_i32(out + opos[t] + 1 + cs[t], (int32_t)dl[t]);
}

unsigned grid_cap(int64_t n) {
    const unsigned g = grid_for(n > 0 ? n : 1, 256);
    return g > 8192 ? 8192 : g;
}

}  // namespace

size_t delta_workspace_bytes(int64_t n) {
    const int64_t nt = n / 2 + 2;   // openers alternate with closers: <= n/2 + 1 tokens
    return (size_t)(4 * n + (n + 1) + 7 * nt + scan_partials_needed(n + 1) + 16 + 64) * sizeof(int64_t);
}

int delta_encode_dev(const uint8_t* X, int64_t n, uint8_t* out, int64_t out_cap, int64_t* out_len,
                     bool* stoi_fail, void* ws, hipStream_t s) {
    *stoi_fail = false;
    *out_len = 0;
    if (n <= 0) return 0;
    const int64_t nt = n / 2 + 2;
    int64_t* p = reinterpret_cast<int64_t*>(ws);
    int64_t* sc = p; p += 64;                 // [0] openers [1] closers [2] commas [3] shift [4] err
    int64_t* lp = p; p += n;
    int64_t* ro = p; p += n;
    int64_t* rc = p; p += n;                  // later: edit marks E
    int64_t* rm = p; p += n;                  // later: max-scan of E
    int64_t* mpos = p; p += n + 1;
    int64_t* opos = p; p += nt;
    int64_t* cpos = p; p += nt;
    int64_t* qpos = p; p += nt;
    int64_t* val = p; p += nt;
    int64_t* hv = p; p += nt;                 // -> previous comma token
    int64_t* dl = p; p += nt;
    int64_t* sh = p; p += nt;
    int64_t* part = p;
    int64_t* csum = hv;                       // hv is consumed by k_dx_shift before the sum lands

    const unsigned g = grid_cap(n), gt = grid_cap(nt);
    int rc_ = dev_set_i64(sc, 8, {0, 0, 0, 0, 0, 0, 0, 0}, s);
    if (rc_) return rc_;
    // last parenthesis strictly before i (negative: none)
    if ((rc_ = dc_last_paren(X, n, lp, part, s))) return rc_;
    hipLaunchKernelGGL(k_dx_flags, dim3(g), dim3(256), 0, s, X, n, (const int64_t*)lp, ro, rc, rm);
    if ((rc_ = dev_excl_sum(ro, ro, n, sc + 0, part, s))) return rc_;
    if ((rc_ = dev_excl_sum(rc, rc, n, sc + 1, part, s))) return rc_;
    if ((rc_ = dev_excl_sum(rm, rm, n, sc + 2, part, s))) return rc_;
    hipLaunchKernelGGL(k_dx_scatter, dim3(g), dim3(256), 0, s, X, n, (const int64_t*)lp, (const int64_t*)ro,
                       (const int64_t*)rc, (const int64_t*)rm, opos, cpos, mpos);
    hipLaunchKernelGGL(k_dx_tokens, dim3(gt), dim3(256), 0, s, X, (const int64_t*)rm, (const int64_t*)opos,
                       (const int64_t*)cpos, (const int64_t*)mpos, qpos, val, hv, nt, sc);
    if ((rc_ = dev_excl_max(hv, hv, nt, nullptr, part, s))) return rc_;
    hipLaunchKernelGGL(k_dx_shift, dim3(gt), dim3(256), 0, s, (const int64_t*)opos, (const int64_t*)qpos,
                       (const int64_t*)val, (const int64_t*)hv, dl, sh, nt);
    if ((rc_ = dev_excl_sum(sh, csum, nt, sc + 3, part, s))) return rc_;
    int64_t* E = rc;
    int64_t* Ex = rm;
    hipLaunchKernelGGL(k_dx_fill, dim3(g), dim3(256), 0, s, E, n, (int64_t)-1);
    hipLaunchKernelGGL(k_dx_mark, dim3(gt), dim3(256), 0, s, (const int64_t*)opos, (const int64_t*)qpos, E, nt);
    if ((rc_ = dev_excl_max(E, Ex, n, nullptr, part, s))) return rc_;
    SCCG_HIP(hipGetLastError());
    int64_t h[5];
    {
        const RbItem it{sc, h, (int)sizeof h};
        if ((rc_ = dev_readback(&it, 1, s))) return rc_;
    }
    if (h[4]) {   // stoi throws: the reference keeps the absolute text
        if (n > out_cap) return SCCG_E_NOMEM;
        SCCG_HIP(hipMemcpyAsync(out, X, (size_t)n, hipMemcpyDeviceToDevice, s));
        *stoi_fail = true;
        *out_len = n;
        return 0;
    }
    const int64_t total = n + h[3];
    if (total > out_cap) return SCCG_E_NOMEM;
    hipLaunchKernelGGL(k_dx_copy, dim3(g), dim3(256), 0, s, X, n, (const int64_t*)E, (const int64_t*)Ex,
                       (const int64_t*)qpos, (const int64_t*)csum, (const int64_t*)sh, out);
    hipLaunchKernelGGL(k_dx_edit, dim3(gt), dim3(256), 0, s, (const int64_t*)opos, (const int64_t*)qpos,
                       (const int64_t*)csum, (const int64_t*)dl, out, nt);
    SCCG_HIP(hipGetLastError());
    *out_len = total;
    return 0;
}
