// scan.hip -- device-wide exclusive scans (reduce-then-scan, three launches).
//
// Used for every compaction offset in the pipeline (FASTA strip, run lists, per-segment and
// per-match text offsets).  Tile = 256 threads x 16 items; block partials are scanned by one
// 256-thread block.  HBM-bound: 8 B read twice + 8 B written per element.
#include "internal.h"

#include <cstring>

namespace {

constexpr int ITEMS = 16;
constexpr int TILE = SCCG_BLOCK * ITEMS;

struct OpSum {
    static __device__ __forceinline__ int64_t id() { return 0; }
    static __device__ __forceinline__ int64_t f(int64_t a, int64_t b) { return a + b; }
};
struct OpMax {
    static __device__ __forceinline__ int64_t id() { return INT64_MIN; }
    static __device__ __forceinline__ int64_t f(int64_t a, int64_t b) { return a > b ? a : b; }
};

template <class Op>
__device__ __forceinline__ int64_t wave_incl(int64_t v) {
    const int lane = lane_id();
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        int64_t o = __shfl_up(v, d, 64);
        if (lane >= d) v = Op::f(v, o);
    }
    return v;
}

// exclusive block scan with arbitrary op; returns exclusive value, *total = block aggregate
template <class Op>
__device__ int64_t block_excl(int64_t v, int64_t* tmp /*17*/, int64_t* total) {
    int64_t incl = wave_incl<Op>(v);
    const int w = wave_in_block(), lane = lane_id(), nw = (int)(blockDim.x >> 6);
    int64_t excl_in_wave = __shfl_up(incl, 1, 64);
    if (lane == 0) excl_in_wave = Op::id();
    if (lane == 63) tmp[w] = incl;
    __syncthreads();
    if (threadIdx.x == 0) {
        int64_t s = Op::id();
        for (int i = 0; i < nw; i++) { int64_t t = tmp[i]; tmp[i] = s; s = Op::f(s, t); }
        tmp[16] = s;
    }
    __syncthreads();
    int64_t r = Op::f(tmp[w], excl_in_wave);
    if (total) *total = tmp[16];
    __syncthreads();
    return r;
}

// Up to two independent scans of the same length share each launch (blockIdx.y picks the array):
// the record line's two block-prefix scans run as three launches instead of six.
struct ScanArrays {
    const int64_t* in[2];
    int64_t* out[2];
    int64_t* total[2];
    int64_t* partial[2];
};

template <class Op>
__global__ __launch_bounds__(SCCG_BLOCK) void k_tile_reduce(ScanArrays a, int64_t n) {
    __shared__ int64_t tmp[17];
    const int64_t* __restrict__ in = a.in[blockIdx.y];
    const int64_t base = (int64_t)blockIdx.x * TILE;
    int64_t acc = Op::id();
#pragma unroll
    for (int i = 0; i < ITEMS; i++) {
        int64_t idx = base + (int64_t)i * SCCG_BLOCK + threadIdx.x;
        if (idx < n) acc = Op::f(acc, in[idx]);
    }
    int64_t tot;
    block_excl<Op>(acc, tmp, &tot);
    if (threadIdx.x == 0) a.partial[blockIdx.y][blockIdx.x] = tot;
}

// Single-block scans: SCCG_SB_T threads (256-thread builds do not wait for a whole free CU beside
// other grids; A/B on the genome bench within noise, so 1024 stays).
#ifndef SCCG_SB_T
#define SCCG_SB_T 1024
#endif
constexpr int SB_T = SCCG_SB_T, PART_PER = 4;
// A short scan (the usual case: a few dozen tile partials, or a few thousand elements) runs in one
// wave or a 256-thread block instead: a 1024-thread block needs a CU with 16 free wave slots, and
// beside another grid (the reconstruction's reference strip) it waited for one -- 72 us of the chr1
// reconstruction's critical path for a 19-element scan (gpurun_out/r05q/dprof).
template <class Op, int T = SB_T>
__global__ __launch_bounds__(T) void k_partials_scan(ScanArrays a, int64_t nb) {
    __shared__ int64_t tmp[17];
    int64_t* __restrict__ partial = a.partial[blockIdx.y];
    int64_t* total = a.total[blockIdx.y];
    int64_t carry = Op::id();
    for (int64_t base = 0; base < nb; base += T * PART_PER) {
        const int64_t i0 = base + (int64_t)threadIdx.x * PART_PER;
        int64_t v[PART_PER], acc = Op::id();
#pragma unroll
        for (int k = 0; k < PART_PER; k++) {
            v[k] = i0 + k < nb ? partial[i0 + k] : Op::id();
            acc = Op::f(acc, v[k]);
        }
        int64_t tot;
        int64_t run = Op::f(carry, block_excl<Op>(acc, tmp, &tot));
#pragma unroll
        for (int k = 0; k < PART_PER; k++) {
            if (i0 + k < nb) partial[i0 + k] = run;
            run = Op::f(run, v[k]);
        }
        carry = Op::f(carry, tot);
    }
    if (threadIdx.x == 0 && total) *total = carry;
}

template <class Op>
__global__ __launch_bounds__(SCCG_BLOCK) void k_tile_scan(ScanArrays a, int64_t n) {
    __shared__ int64_t tmp[17];
    const int64_t* __restrict__ in = a.in[blockIdx.y];
    int64_t* __restrict__ out = a.out[blockIdx.y];
    // each thread owns ITEMS consecutive elements
    const int64_t base = (int64_t)blockIdx.x * TILE + (int64_t)threadIdx.x * ITEMS;
    int64_t v[ITEMS];
    int64_t acc = Op::id();
#pragma unroll
    for (int i = 0; i < ITEMS; i++) {
        v[i] = (base + i < n) ? in[base + i] : Op::id();
        acc = Op::f(acc, v[i]);
    }
    int64_t ex = block_excl<Op>(acc, tmp, nullptr);
    int64_t run = Op::f(a.partial[blockIdx.y][blockIdx.x], ex);
#pragma unroll
    for (int i = 0; i < ITEMS; i++) {
        if (base + i < n) out[base + i] = run;
        run = Op::f(run, v[i]);
    }
}

// small inputs (<= 16 Ki elements): one 256-thread block, one launch; a thread owns up to 64
// consecutive elements, reduced 16 at a time (the 16 loads issued together), then re-read
// (L2-hot) for the prefixes
constexpr int SMALL_PER = 16, SMALL_MAX = 16384;   // (<= 64 elements per thread at 256 threads)
template <class Op, int T = SB_T>
__global__ __launch_bounds__(T) void k_small_scan(ScanArrays a, int64_t n) {
    __shared__ int64_t tmp[17];
    const int64_t* __restrict__ in = a.in[blockIdx.y];
    int64_t* __restrict__ out = a.out[blockIdx.y];
    int64_t* total = a.total[blockIdx.y];
    const int64_t per = (n + T - 1) / T, base = (int64_t)threadIdx.x * per;
    int64_t acc = Op::id();
    for (int64_t g = 0; g < per; g += SMALL_PER) {
        int64_t v[SMALL_PER];
#pragma unroll
        for (int i = 0; i < SMALL_PER; i++) v[i] = (g + i < per && base + g + i < n) ? in[base + g + i] : Op::id();
#pragma unroll
        for (int i = 0; i < SMALL_PER; i++) acc = Op::f(acc, v[i]);
    }
    int64_t tot;
    int64_t run = block_excl<Op>(acc, tmp, &tot);
    for (int64_t g = 0; g < per; g += SMALL_PER) {
        int64_t v[SMALL_PER];
#pragma unroll
        for (int i = 0; i < SMALL_PER; i++) v[i] = (g + i < per && base + g + i < n) ? in[base + g + i] : Op::id();
#pragma unroll
        for (int i = 0; i < SMALL_PER; i++) {
            if (g + i < per && base + g + i < n) out[base + g + i] = run;
            run = Op::f(run, v[i]);
        }
    }
    if (threadIdx.x == 0 && total) *total = tot;
}

template <class Op>
int scan_impl(const ScanArrays& a, int m, int64_t n, hipStream_t s) {
    if (n <= 0) {
        for (int i = 0; i < m; i++)
            if (a.total[i]) {
                const int rc = dev_set_i64(a.total[i], 1, {0}, s);
                if (rc) return rc;
            }
        return 0;
    }
    if (n <= 64 * SMALL_PER) {
        hipLaunchKernelGGL((k_small_scan<Op, 64>), dim3(1, m), dim3(64), 0, s, a, n);
        SCCG_HIP(hipGetLastError());
        return 0;
    }
    if (n <= 256 * SMALL_PER) {
        hipLaunchKernelGGL((k_small_scan<Op, 256>), dim3(1, m), dim3(256), 0, s, a, n);
        SCCG_HIP(hipGetLastError());
        return 0;
    }
    if (n <= SMALL_MAX) {
        hipLaunchKernelGGL(k_small_scan<Op>, dim3(1, m), dim3(SB_T), 0, s, a, n);
        SCCG_HIP(hipGetLastError());
        return 0;
    }
    const int64_t nb = (n + TILE - 1) / TILE;
    hipLaunchKernelGGL(k_tile_reduce<Op>, dim3((unsigned)nb, m), dim3(SCCG_BLOCK), 0, s, a, n);
    if (nb <= 64 * PART_PER) hipLaunchKernelGGL((k_partials_scan<Op, 64>), dim3(1, m), dim3(64), 0, s, a, nb);
    else if (nb <= 256 * PART_PER) hipLaunchKernelGGL((k_partials_scan<Op, 256>), dim3(1, m), dim3(256), 0, s, a, nb);
    else hipLaunchKernelGGL(k_partials_scan<Op>, dim3(1, m), dim3(SB_T), 0, s, a, nb);
    hipLaunchKernelGGL(k_tile_scan<Op>, dim3((unsigned)nb, m), dim3(SCCG_BLOCK), 0, s, a, n);
    SCCG_HIP(hipGetLastError());
    return 0;
}

template <class Op>
int scan_one(const int64_t* in, int64_t* out, int64_t n, int64_t* d_total, int64_t* d_partial, hipStream_t s) {
    const ScanArrays a{{in, in}, {out, out}, {d_total, d_total}, {d_partial, d_partial}};
    return scan_impl<Op>(a, 1, n, s);
}

struct Vals8 {
    int64_t v[8];
};
__global__ void k_set_i64(int64_t* p, int n, Vals8 v) {
    if ((int)threadIdx.x < n) p[threadIdx.x] = v.v[threadIdx.x];
}
struct Vals8i {
    int32_t v[8];
};
__global__ void k_set_i32(int32_t* p, int n, Vals8i v) {
    if ((int)threadIdx.x < n) p[threadIdx.x] = v.v[threadIdx.x];
}

struct Bytes16 {
    uint8_t v[16];
};
__global__ void k_set_u8(uint8_t* p, int n, Bytes16 v) {
    if ((int)threadIdx.x < n) p[threadIdx.x] = v.v[threadIdx.x];
}

}  // namespace

namespace {
// dst = pre, src[0, n), post
__global__ void k_put_framed(uint8_t* __restrict__ dst, const uint8_t* __restrict__ src, int64_t n, uint8_t pre,
                             uint8_t post) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n + 2; i += (int64_t)gridDim.x * blockDim.x)
        dst[i] = i == 0 ? pre : (i == n + 1 ? post : src[i - 1]);
}
}  // namespace

int dev_put_framed(uint8_t* dst, const uint8_t* src, int64_t n, char pre, char post, hipStream_t s) {
    const unsigned g = grid_for(n + 2, 256) > 1024 ? 1024 : grid_for(n + 2, 256);
    hipLaunchKernelGGL(k_put_framed, dim3(g), dim3(256), 0, s, dst, src, n, (uint8_t)pre, (uint8_t)post);
    SCCG_HIP(hipGetLastError());
    return 0;
}

namespace {
// out[0, hlen) = hdr, out[hlen] = '\n', out[total - 1] = '\n'
__global__ void k_put_frame(uint8_t* __restrict__ out, const uint8_t* __restrict__ hdr, int64_t hlen, int64_t total) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i <= hlen; i += (int64_t)gridDim.x * blockDim.x)
        out[i] = i < hlen ? hdr[i] : (uint8_t)'\n';
    if (blockIdx.x == 0 && threadIdx.x == 0) out[total - 1] = '\n';
}
}  // namespace

int dev_put_frame(uint8_t* out, const uint8_t* hdr, int64_t hlen, int64_t total, hipStream_t s) {
    const unsigned g = grid_for(hlen + 1, 256) > 64 ? 64 : grid_for(hlen + 1, 256);
    hipLaunchKernelGGL(k_put_frame, dim3(g), dim3(256), 0, s, out, hdr, hlen, total);
    SCCG_HIP(hipGetLastError());
    return 0;
}

int dev_put_bytes(uint8_t* p, const char* bytes, int n, hipStream_t s) {
    Bytes16 v{};
    if (n > 16) return SCCG_E_INTERNAL;
    for (int i = 0; i < n; i++) v.v[i] = (uint8_t)bytes[i];
    hipLaunchKernelGGL(k_set_u8, dim3(1), dim3(64), 0, s, p, n, v);
    SCCG_HIP(hipGetLastError());
    return 0;
}

// Stream-ordered writes of up to 8 scalars: the values travel as kernel arguments, so no host
// buffer has to outlive the call (a hipMemcpyAsync from a stack temporary would).
int dev_set_i64(int64_t* p, int n, std::initializer_list<int64_t> vals, hipStream_t s) {
    Vals8 v{};
    int i = 0;
    for (int64_t x : vals) if (i < 8) v.v[i++] = x;
    hipLaunchKernelGGL(k_set_i64, dim3(1), dim3(64), 0, s, p, n < i ? n : i, v);
    SCCG_HIP(hipGetLastError());
    return 0;
}
int dev_set_i32(int32_t* p, int n, std::initializer_list<int32_t> vals, hipStream_t s) {
    Vals8i v{};
    int i = 0;
    for (int32_t x : vals) if (i < 8) v.v[i++] = x;
    hipLaunchKernelGGL(k_set_i32, dim3(1), dim3(64), 0, s, p, n < i ? n : i, v);
    SCCG_HIP(hipGetLastError());
    return 0;
}

int64_t scan_partials_needed(int64_t n) { return (n + TILE - 1) / TILE + 1; }

int dev_excl_sum(const int64_t* in, int64_t* out, int64_t n, int64_t* d_total, int64_t* d_partial,
                 hipStream_t s) {
    return scan_one<OpSum>(in, out, n, d_total, d_partial, s);
}

int dev_excl_sum2(const int64_t* in0, int64_t* out0, int64_t* d_total0, const int64_t* in1, int64_t* out1,
                  int64_t* d_total1, int64_t n, int64_t* d_partial, hipStream_t s) {
    const int64_t np = scan_partials_needed(n);
    const ScanArrays a{{in0, in1}, {out0, out1}, {d_total0, d_total1}, {d_partial, d_partial + np}};
    return scan_impl<OpSum>(a, 2, n, s);
}

int dev_excl_max(const int64_t* in, int64_t* out, int64_t n, int64_t* d_total, int64_t* d_partial,
                 hipStream_t s) {
    return scan_one<OpMax>(in, out, n, d_total, d_partial, s);
}

// ---------------------------------------------------------------------------------------------
// Low-latency readback of a few small device values.  One single-wave kernel copies them into
// pinned, fine-grained host memory and then publishes a sequence number there with a system-scope
// release; the host spins on that number.  Compared with hipMemcpyAsync + hipStreamSynchronize
// this has no copy-engine command and no interrupt wake-up on the host's critical path (a
// stream-synchronise round trip costs 20-45 us between kernels here, the spin a few).
// ---------------------------------------------------------------------------------------------
namespace {
constexpr int RB_MAX = 8;
constexpr int RB_BYTES = 4096 - 64;
struct RbArgs {
    const uint8_t* src[RB_MAX];
    int32_t off[RB_MAX];
    int32_t bytes[RB_MAX];
    int32_t n;
};
__global__ void k_readback(RbArgs a, uint8_t* __restrict__ host, unsigned long long* flag, unsigned long long seq) {
    for (int i = 0; i < a.n; i++) {
        const uint8_t* src = a.src[i];
        uint8_t* dst = host + a.off[i];
        const int nb = a.bytes[i];
        if ((((uintptr_t)src) & 3) == 0 && (nb & 3) == 0) {
            for (int b = (int)threadIdx.x; b < nb / 4; b += (int)blockDim.x)
                reinterpret_cast<uint32_t*>(dst)[b] = reinterpret_cast<const uint32_t*>(src)[b];
        } else {
            for (int b = (int)threadIdx.x; b < nb; b += (int)blockDim.x) dst[b] = src[b];
        }
    }
    __threadfence_system();
    __syncthreads();
    if (threadIdx.x == 0) __hip_atomic_store(flag, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}
struct RbHost {
    uint8_t* buf = nullptr;   // [0, 64): flag; [64, 4096): data
    uint8_t* dbuf = nullptr;  // device view
    unsigned long long seq = 0;
};
thread_local RbHost g_rb;
}  // namespace

int dev_readback(const RbItem* items, int n, hipStream_t s) {
    if (n <= 0) return 0;
    if (n > RB_MAX) return SCCG_E_INVALID;
    if (!g_rb.buf) {
        void* p = nullptr;
        SCCG_HIP(hipHostMalloc(&p, 4096, hipHostMallocMapped | hipHostMallocCoherent | hipHostMallocPortable));
        void* dp = nullptr;
        SCCG_HIP(hipHostGetDevicePointer(&dp, p, 0));
        g_rb.buf = static_cast<uint8_t*>(p);
        g_rb.dbuf = static_cast<uint8_t*>(dp);
        *reinterpret_cast<volatile unsigned long long*>(g_rb.buf) = 0;
    }
    RbArgs a{};
    int off = 0;
    for (int i = 0; i < n; i++) {
        if (items[i].bytes < 0 || off + items[i].bytes > RB_BYTES) return SCCG_E_INVALID;
        a.src[i] = static_cast<const uint8_t*>(items[i].src);
        a.off[i] = off;
        a.bytes[i] = items[i].bytes;
        off += (items[i].bytes + 7) & ~7;
    }
    a.n = n;
    const unsigned long long seq = ++g_rb.seq;
    unsigned long long* flag = reinterpret_cast<unsigned long long*>(g_rb.buf);
    hipLaunchKernelGGL(k_readback, dim3(1), dim3(64), 0, s, a, g_rb.dbuf + 64,
                       reinterpret_cast<unsigned long long*>(g_rb.dbuf), seq);
    SCCG_HIP(hipGetLastError());
    for (uint64_t it = 1;; it++) {
        if (__atomic_load_n(flag, __ATOMIC_ACQUIRE) == seq) break;
        if ((it & 4095) == 0) {
            // the stream failed, or drained without the flag arriving: fall back to a full wait
            const hipError_t e = hipStreamQuery(s);
            if (e != hipErrorNotReady) {
                SCCG_HIP(e == hipSuccess ? hipStreamSynchronize(s) : e);
                if (__atomic_load_n(flag, __ATOMIC_ACQUIRE) != seq) {
                    return sccg_hip_fail(hipErrorUnknown, "readback flag not raised by a finished stream", __FILE__,
                                         __LINE__);
                }
                break;
            }
        }
        __builtin_ia32_pause();
    }
    for (int i = 0; i < n; i++) memcpy(items[i].dst, g_rb.buf + 64 + a.off[i], (size_t)items[i].bytes);
    return 0;
}
