// common.h -- device helpers shared by the SCCG kernels (gfx950, wave64).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#define SCCG_WAVE 64
#define SCCG_BLOCK 256

// ---------------------------------------------------------------------------------------------
// byte classes (C locale, as the reference's ::isspace / islower / toupper)
// ---------------------------------------------------------------------------------------------
__host__ __device__ __forceinline__ bool c_isspace(uint8_t c) { return c == ' ' || (c >= 9 && c <= 13); }
__host__ __device__ __forceinline__ bool c_islower(uint8_t c) { return c >= 'a' && c <= 'z'; }
__host__ __device__ __forceinline__ uint8_t c_toupper(uint8_t c) { return c_islower(c) ? (uint8_t)(c - 32) : c; }
__host__ __device__ __forceinline__ uint8_t c_tolower(uint8_t c) { return (c >= 'A' && c <= 'Z') ? (uint8_t)(c + 32) : c; }
// 2-bit code of an (uppercase) nucleotide, 4 for every other byte
__host__ __device__ __forceinline__ uint32_t base2(uint8_t c) {
    return c == 'A' ? 0u : c == 'C' ? 1u : c == 'G' ? 2u : c == 'T' ? 3u : 4u;
}

// k-mer key: pure A/C/G/T k-mers (k <= 15) -> their 2k-bit code (< 2^30); k-mers holding any
// other byte -> 0x80000000 | 31-bit FNV-1a of the bytes.  Equal pure keys <=> equal bytes; equal
// "exotic" keys must be confirmed by a byte compare.
#define KEY_EXOTIC 0x80000000u
__host__ __device__ __forceinline__ uint32_t exotic_key(const uint8_t* s, int k) {
    uint32_t h = 2166136261u;
    for (int i = 0; i < k; i++) { h ^= s[i]; h *= 16777619u; }
    return KEY_EXOTIC | (h & 0x7fffffffu);
}
__host__ __device__ __forceinline__ uint32_t kmer_key(const uint8_t* s, int k) {
    uint32_t code = 0;
    for (int i = 0; i < k; i++) {
        uint32_t b = base2(s[i]);
        if (b > 3) return exotic_key(s, k);
        code = (code << 2) | b;
    }
    return code;
}
__host__ __device__ __forceinline__ uint32_t slot_hash(uint32_t key, int bits) {
    return (key * 0x9E3779B1u) >> (32 - bits);
}
__host__ __device__ __forceinline__ int ndigits_u32(uint32_t v) {
    int n = 1;
    while (v >= 10) { v /= 10; n++; }
    return n;
}
// decimal length of a signed int, as operator<< / to_string print it
__host__ __device__ __forceinline__ int ndigits_i32(int32_t v) {
    return v < 0 ? 1 + ndigits_u32((uint32_t)0 - (uint32_t)v) : ndigits_u32((uint32_t)v);
}
__device__ __forceinline__ int write_i32(uint8_t* dst, int32_t v) {
    uint32_t u = v < 0 ? (uint32_t)0 - (uint32_t)v : (uint32_t)v;
    int n = ndigits_u32(u) + (v < 0);
    int w = n;
    do { dst[--w] = (uint8_t)('0' + u % 10); u /= 10; } while (u);
    if (v < 0) dst[0] = '-';
    return n;
}

// ---------------------------------------------------------------------------------------------
// Packed ("walk") k-mer keys: a pure A/C/G/T k-mer's key is its 2-bit codes packed first base
// LOWEST (bits 2i..2i+1 = base i), so the keys of every k-mer in a run of bytes are shifts of one
// packed word computed 4 bytes at a time (SWAR); a k-mer holding any other byte gets exotic_key()
// (high bit set, confirmed by a byte compare).  Equal pure keys <=> equal bytes.  Each kernel
// uses one convention for all the keys it compares (walk, full sweeps, local segments).
// ---------------------------------------------------------------------------------------------
// 4 bytes -> their 2-bit codes in 8 bits (byte i at bits 2i), and `diff` nonzero in exactly the
// bytes that are not A/C/G/T: code = ((c >> 1) ^ (c >> 2)) & 3 maps A,C,G,T -> 0,1,2,3, and a
// byte-permute of "ACGT" by the codes rebuilds the byte iff it was one of them.
__device__ __forceinline__ uint32_t swar_codes(uint32_t w, uint32_t& diff) {
    const uint32_t c = ((w >> 1) ^ (w >> 2)) & 0x03030303u;
    diff = __builtin_amdgcn_perm(0x54474341u, 0x54474341u, c) ^ w;
    const uint32_t p = c | (c >> 6);
    return (p | (p >> 12)) & 0xffu;
}
// bit i set <=> byte i of `diff` is nonzero
__device__ __forceinline__ uint32_t nz_bytes(uint32_t diff) {
    const uint32_t nz = ((((diff & 0x7f7f7f7fu) + 0x7f7f7f7fu) | diff) & 0x80808080u) >> 7;
    return (nz | (nz >> 7) | (nz >> 14) | (nz >> 21)) & 0xfu;
}
// ND consecutive words -> packed codes (byte i at bits 2i) and the non-ACGT byte mask
template <int ND>
__device__ __forceinline__ void pack_codes(const uint32_t (&w)[ND], uint64_t& code, uint32_t& bad) {
    uint32_t d[ND], acc = 0;
    code = 0;
#pragma unroll
    for (int i = 0; i < ND; i++) {
        code |= (uint64_t)swar_codes(w[i], d[i]) << (8 * i);
        acc |= d[i];
    }
    bad = 0;
    if (acc) {   // rare: some byte is not A/C/G/T
#pragma unroll
        for (int i = 0; i < ND; i++) bad |= nz_bytes(d[i]) << (4 * i);
    }
}
// ND words from an arbitrary (global or LDS) address: ND+1 aligned dword loads.  The aligned base
// is formed by pointer arithmetic on p (not through an integer): the compiler then keeps p's address
// space and emits global loads; a pointer rebuilt from an integer is generic, and FLAT loads also
// count against lgkmcnt, so every later LDS wait would wait for the HBM load too.
template <int ND>
__device__ __forceinline__ void loadw(const uint8_t* p, uint32_t (&o)[ND]) {
    const uint32_t sh = (uint32_t)((uintptr_t)p & 3);
    const uint32_t* w = reinterpret_cast<const uint32_t*>(p - sh);
    uint32_t v[ND + 1];
#pragma unroll
    for (int i = 0; i <= ND; i++) v[i] = w[i];
#pragma unroll
    for (int i = 0; i < ND; i++) o[i] = __builtin_amdgcn_alignbyte(v[i + 1], v[i], sh);
}
// scalar form (any k <= 15)
__device__ __forceinline__ uint32_t walk_key(const uint8_t* s, int k) {
    uint32_t code = 0;
    for (int i = 0; i < k; i++) {
        const uint32_t b = base2(s[i]);
        if (b > 3) return exotic_key(s, k);
        code |= b << (2 * i);
    }
    return code;
}

// ---------------------------------------------------------------------------------------------
// wave64 primitives
// ---------------------------------------------------------------------------------------------
__device__ __forceinline__ int lane_id() { return (int)(threadIdx.x & 63); }
__device__ __forceinline__ int wave_in_block() { return (int)(threadIdx.x >> 6); }

// Orders LDS traffic between the lanes of ONE wave (other waves of the block run their own
// loops, so no workgroup barrier is possible there).
__device__ __forceinline__ void wave_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

template <typename T>
__device__ __forceinline__ T wave_incl_add(T v) {
    const int lane = lane_id();
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        T o = __shfl_up(v, d, 64);
        if (lane >= d) v += o;
    }
    return v;
}
// 32-bit inclusive wave scan on DPP (six v_add_u32_dpp, against ~36 VALU and six ds_bpermute for
// the shuffle ladder above): row_shr 1/2/4/8 inside each 16-lane row (bound_ctrl: lanes shifted in
// from outside the row add 0), then row 0's total into row 1 and row 2's into row 3 (row_bcast:15),
// then rows 0-1's into rows 2-3 (row_bcast:31).  Needs the whole wave active.  Packed counters
// scan field by field as long as no field's total carries into the next.
__device__ __forceinline__ uint32_t wave_incl_add_dpp(uint32_t v) {
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x111, 0xf, 0xf, true);
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x112, 0xf, 0xf, true);
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x114, 0xf, 0xf, true);
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x118, 0xf, 0xf, true);
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x142, 0xa, 0xf, false);
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x143, 0xc, 0xf, false);
    return v;
}
template <typename T>
__device__ __forceinline__ T wave_sum(T v) {
#pragma unroll
    for (int d = 32; d > 0; d >>= 1) v += __shfl_xor(v, d, 64);
    return v;
}
template <typename T>
__device__ __forceinline__ T wave_max(T v) {
#pragma unroll
    for (int d = 32; d > 0; d >>= 1) { T o = __shfl_xor(v, d, 64); v = o > v ? o : v; }
    return v;
}
template <typename T>
__device__ __forceinline__ T wave_min(T v) {
#pragma unroll
    for (int d = 32; d > 0; d >>= 1) { T o = __shfl_xor(v, d, 64); v = o < v ? o : v; }
    return v;
}
__device__ __forceinline__ int first_lane(unsigned long long m) { return m ? __ffsll((long long)m) - 1 : 64; }
// wave-uniform copies (SGPR): a value every lane agrees on, and lane l's value
__device__ __forceinline__ int32_t uni(int32_t v) { return __builtin_amdgcn_readfirstlane(v); }
__device__ __forceinline__ int32_t lane_val(int32_t v, int l) { return __builtin_amdgcn_readlane(v, l); }
__device__ __forceinline__ uint32_t lane_val(uint32_t v, int l) { return (uint32_t)__builtin_amdgcn_readlane((int32_t)v, l); }

// exclusive block scan (sum) for a 256-thread block; `tmp` = 5 LDS slots
template <typename T>
__device__ __forceinline__ T block_excl_add(T v, T* tmp, T* total) {
    T incl = wave_incl_add(v);
    const int w = wave_in_block(), lane = lane_id();
    if (lane == 63) tmp[w] = incl;
    __syncthreads();
    if (threadIdx.x == 0) {
        T s = 0;
        for (int i = 0; i < (int)(blockDim.x >> 6); i++) { T t = tmp[i]; tmp[i] = s; s += t; }
        tmp[4] = s;
    }
    __syncthreads();
    T r = incl - v + tmp[w];
    if (total) *total = tmp[4];
    __syncthreads();
    return r;
}

// ---------------------------------------------------------------------------------------------
// HIP error plumbing (host side)
// ---------------------------------------------------------------------------------------------
#define SCCG_HIP(expr)                                              \
    do {                                                            \
        hipError_t e_ = (expr);                                     \
        if (e_ != hipSuccess) return sccg_hip_fail(e_, #expr, __FILE__, __LINE__); \
    } while (0)

int sccg_hip_fail(hipError_t e, const char* what, const char* file, int line);

static inline unsigned grid_for(int64_t n, int per_block) {
    int64_t g = (n + per_block - 1) / per_block;
    return (unsigned)(g < 1 ? 1 : g);
}
