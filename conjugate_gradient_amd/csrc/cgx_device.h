// cgx_device.h -- internal to libcgx: device and host helpers shared by the
// kernel files (cgx_matvec.hip, cgx_vector.hip, cgx_poisson.hip,
// cgx_ref_f32.hip, cgx_symv.hip).  Not part of the C ABI (include/cgx.h).
#pragma once

#include "cgx_kernels.h"

#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <mutex>

namespace cgx {

typedef double d2 __attribute__((ext_vector_type(2)));

constexpr int kNT = 256;  // threads per block for the fp64 kernels

// CG's alpha = r.r / p.Ap and beta = r.r_new / r.r_old, fp64.  A zero
// denominator under a numerator that has underflowed too (|num| below the
// smallest normal double, 0 included) means the iteration has converged
// exactly -- r = 0, or, in a fixed-count run that goes on long past
// convergence, r.r and p.Ap have sunk into the subnormals, where their
// rounding is noise: that is CG's "lucky breakdown", and the ratio is 0, so x
// stays at the solution and r, p stay 0 instead of turning into NaN.  Every
// other pair gives the plain quotient, bit for bit -- in particular a normal
// r.r over p.Ap = 0 (an A that is not positive definite), which is a real
// breakdown and shows up as Inf / NaN exactly as the reference's division
// would (test_indefinite_breakdown_is_not_hidden).  (An SPD A keeps p.Ap >=
// lambda_min |p|^2 ~ lambda_min r.r, nonzero while r.r is normal.)
// CGX_F32_REF keeps the reference's float division as it is
// (serialConjugate.c:220,239).
// A system-scope load (sc0 sc1): coherent with another device's writes made
// visible by its system-scope release (the one-process multi-shard exchange
// reads peers' memory this way; cgx_kernels.h PeerTable).
template <typename T>
__device__ __forceinline__ T load_sys(const T *p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

// The cnt (<= 64) per-shard partials src.p[q], one per lane, loaded together
// (one round trip, not cnt): lanes past cnt hold 0.
template <typename T>
__device__ __forceinline__ T peer_lane_load(const PeerTable &src, int cnt) {
    const int lane = threadIdx.x & 63;
    return lane < cnt ? load_sys(reinterpret_cast<const T *>(src.p[lane])) : T(0);
}
__device__ __forceinline__ double readlane_f64(double v, int lane) {
    const uint64_t b = __builtin_bit_cast(uint64_t, v);
    const uint32_t lo = __builtin_amdgcn_readlane((uint32_t)b, lane), hi = __builtin_amdgcn_readlane((uint32_t)(b >> 32), lane);
    return __builtin_bit_cast(double, ((uint64_t)hi << 32) | lo);
}
// The rank-order sum x_0 + x_1 + ... of the lanes' values (wave-uniform
// result, the same adds in the same order as a sequential loop).
__device__ __forceinline__ double lane_sum_ordered_f64(double x, int cnt) {
#pragma clang fp contract(off)
    double v = readlane_f64(x, 0);
    for (int q = 1; q < cnt; ++q) v = v + readlane_f64(x, q);
    return v;
}

// PeerSum (cgx_kernels.h): the cnt partials in rank order, computed by every
// wave (the loads go out with the kernel's first vector loads; no barrier,
// no LDS); block 0's thread 0 stores it for later kernels and the host.
__device__ __forceinline__ double peer_sum_wave(const PeerSum &c) {
    const double v = lane_sum_ordered_f64(peer_lane_load<double>(c.src, c.cnt), c.cnt);
    if (blockIdx.x == 0 && threadIdx.x == 0) *c.out = v;
    return v;
}

// PeerSumF32: parallel_cg.c's MPI_Allreduce (MPICH 3.3's recursive doubling)
// of the cnt float partials, by every wave (all 64 lanes active): lane q
// loads partial q, pairs (2q, 2q+1) for q < rem combine first, then the
// pairwise tree over pof2 values -- k_combine_peers<float>'s adds in its
// order; wave-uniform result; block 0's thread 0 stores it.
__device__ __forceinline__ float peer_sum_mpich_f32(const PeerSumF32 &c) {
#pragma clang fp contract(off)
    const int lane = threadIdx.x & 63;
    const float x = peer_lane_load<float>(c.src, c.cnt);
    int pof2 = 1;
    while (pof2 * 2 <= c.cnt) pof2 *= 2;
    const int rem = c.cnt - pof2;
    const float a = __shfl(x, lane < rem ? 2 * lane : (lane + rem) & 63, 64);
    const float b = __shfl(x, (2 * lane + 1) & 63, 64);
    float v = lane < rem ? a + b : a;
    for (int d = 1; d < pof2; d *= 2) {
        const float w = __shfl(v, (lane + d) & 63, 64);
        if (lane % (2 * d) == 0 && lane + d < pof2) v = v + w;
    }
    const float r = __shfl(v, 0, 64);
    if (blockIdx.x == 0 && threadIdx.x == 0) *c.out = r;
    return r;
}

__device__ __forceinline__ double cg_ratio(double num, double den) {
    return (den != 0.0 || !(__builtin_fabs(num) < 0x1p-1022)) ? num / den : 0.0;
}

__device__ __forceinline__ double wave_sum(double v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}

// Sum `v` over all threads of the grid.  Each block stores its total in
// partials[blockIdx.x]; the last block to arrive sums the partials in index
// order and writes *out.  Deterministic for a fixed grid.
//
// Hand-off (kHandoffNote; cdna_hip_programming.md Guideline 16, Recipe R1,
// the write-through form): the partial is stored write-through (8-B
// agent-scope atomic store = sc1), the storing lane drains it (s_waitcnt
// vmcnt(0)) before its relaxed agent-scope ticket add, and the block whose
// add returns gridDim-1 reads every partial with sc1 loads (agent-scope
// atomic loads).
//
// kHandoffNote -- why the producer has no release.  In the C++/HIP memory
// model a relaxed store followed by a relaxed RMW publishes nothing; what
// makes this hand-off correct is gfx950's implementation, which the guide's
// Recipe R1 states as the rule: a payload stored write-through (sc1: past
// this XCD's L2 to the coherence point) and drained by EVERY storing wave
// before the signal "needs no release fence", and a consumer whose every load
// of the payload is an sc1 load needs no L1 invalidate.  Here the payload is
// the partial (an agent-scope atomic store) or, in k_update_xrp_f64 and the
// F32_REF matVec + vecVec, r / Ap stored with 16-B sc1 buffer stores by every
// wave, each wave draining (vmcnt(0)) before the block barrier that precedes
// the ticket.  An agent-scope release on the ticket would add a buffer_wbl2
// (write-back of the whole L2's dirty lines) per block: measured 378 vs 283 us
// on a 537 MB k_update_r (round 1), for no change in what the consumer reads.
// The rule holds for gfx950 (the only target this library builds for); a
// build for another part stops here instead of compiling a hand-off whose
// correctness would rest on that part's cache policy.
#if defined(__HIP_DEVICE_COMPILE__) && !defined(__gfx950__)
#error "cgx: the write-through reduction hand-off (kHandoffNote) is validated on gfx950 only"
#endif
template <int NT = kNT>
__device__ __forceinline__ void grid_sum_last_block(double v, double *partials, unsigned *ticket,
                                                    double *out, bool add_to_out = false) {
    __shared__ double red[NT / 64];
    __shared__ int is_last;
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    v = wave_sum(v);
    if (lane == 0) red[wid] = v;
    __syncthreads();
    if (gridDim.x == 1) {
        // one block (n <= 2048 in the vector kernels): no hand-off through
        // memory, two dependent round trips fewer (fixed-count iterations
        // 5-7 % faster at N=512-2048, profiles/r01_ab_one_block_reduce.txt).
        // The same bits as the hand-off, which adds the block's sum to 0.0
        // (so a -0 sum comes out +0 there too).
        if (threadIdx.x == 0) {
            double t = red[0];
#pragma unroll
            for (int w = 1; w < NT / 64; ++w) t += red[w];
            t = 0.0 + t;
            *out = add_to_out ? *out + t : t;
        }
        return;
    }
    if (threadIdx.x == 0) {
        double t = red[0];
#pragma unroll
        for (int w = 1; w < NT / 64; ++w) t += red[w];
        __hip_atomic_store(partials + blockIdx.x, t, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        const unsigned prev = __hip_atomic_fetch_add(ticket, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        is_last = (prev == gridDim.x - 1);
    }
    __syncthreads();
    if (!is_last) return;
    // Order the partial loads below after the ticket (acquire at agent scope,
    // once per kernel in this one block; it also keeps the compiler from
    // hoisting the loads).  The producer side has no release: see
    // kHandoffNote below for why the hand-off is correct on gfx950 and what a
    // release would cost.
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    // all of this thread's partials in flight at once (grid <= 8192 = 32 * NT)
    double s = 0.0;
    for (unsigned i0 = threadIdx.x; i0 < gridDim.x; i0 += 8 * NT) {
        double pv[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) {
            const unsigned i = i0 + u * NT;
            pv[u] = (i < gridDim.x) ? __hip_atomic_load(partials + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : 0.0;
        }
#pragma unroll
        for (int u = 0; u < 8; ++u)
            if (i0 + u * NT < gridDim.x) s += pv[u];
    }
    s = wave_sum(s);
    if (lane == 0) red[wid] = s;
    __syncthreads();
    if (threadIdx.x == 0) {
        double t = red[0];
#pragma unroll
        for (int w = 1; w < NT / 64; ++w) t += red[w];
        *out = add_to_out ? *out + t : t;
        __hip_atomic_store(ticket, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
}

// grid_sum_last_block's hand-off, but the last block keeps going: returns
// true (block-uniform) in the block that summed the partials, with the total
// in `total` for every thread of it; *out gets the total as well.  The bytes
// the other blocks wrote in this launch are visible to that block only if
// they were stored write-through (sc1) and are loaded with sc1 loads
// (cdna_hip_programming.md Guideline 16, the one-counter row).
__device__ __forceinline__ bool grid_sum_keep_last(double v, double *partials, unsigned *ticket, double *out,
                                                   double &total) {
    __shared__ double red[kNT / 64];
    __shared__ int is_last;
    __shared__ double tot;
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    v = wave_sum(v);
    if (lane == 0) red[wid] = v;
    __syncthreads();
    if (gridDim.x == 1) {  // the same bits as the hand-off below (which adds to 0.0)
        if (threadIdx.x == 0) {
            double t = red[0];
#pragma unroll
            for (int w = 1; w < kNT / 64; ++w) t += red[w];
            tot = 0.0 + t;
            *out = tot;
        }
        __syncthreads();
        total = tot;
        return true;
    }
    if (threadIdx.x == 0) {
        double t = red[0];
#pragma unroll
        for (int w = 1; w < kNT / 64; ++w) t += red[w];
        __hip_atomic_store(partials + blockIdx.x, t, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        const unsigned prev = __hip_atomic_fetch_add(ticket, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        is_last = (prev == gridDim.x - 1);
    }
    __syncthreads();
    if (!is_last) return false;
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    double s = 0.0;
    for (unsigned i0 = threadIdx.x; i0 < gridDim.x; i0 += 8 * kNT) {
        double pv[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) {
            const unsigned i = i0 + u * kNT;
            pv[u] = (i < gridDim.x) ? __hip_atomic_load(partials + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : 0.0;
        }
#pragma unroll
        for (int u = 0; u < 8; ++u)
            if (i0 + u * kNT < gridDim.x) s += pv[u];
    }
    s = wave_sum(s);
    __syncthreads();  // red[] is reused
    if (lane == 0) red[wid] = s;
    __syncthreads();
    if (threadIdx.x == 0) {
        double t = red[0];
#pragma unroll
        for (int w = 1; w < kNT / 64; ++w) t += red[w];
        tot = t;
        *out = t;
        __hip_atomic_store(ticket, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    __syncthreads();
    total = tot;
    return true;
}

// CGX_PHASES timestamps (cgx_kernels.h kTsSlot): ts_start after a kernel's
// gate, ts_end at every block-uniform exit reached by all of the block's
// threads (one extra barrier, then lane 0 of the block stores its exit time).
__device__ __forceinline__ void ts_start(int64_t *ts) {
    if (ts && blockIdx.x == 0 && threadIdx.x == 0) ts[0] = wall_clock64();
}
__device__ __forceinline__ void ts_end(int64_t *ts) {
    if (!ts) return;
    __syncthreads();
    if (threadIdx.x == 0 && blockIdx.x < (unsigned)kTsMaxBlocks) ts[1 + blockIdx.x] = wall_clock64();
}

__device__ __forceinline__ d2 ld2(const double *p) { return *reinterpret_cast<const d2 *>(p); }
__device__ __forceinline__ void st2(double *p, d2 v) { *reinterpret_cast<d2 *>(p) = v; }

// Stream policy of the vector kernels (VP): 0 plain, 1 non-temporal stores,
// 2 non-temporal loads and stores (default: -8 % time on the Poisson
// vectors, 537 MB each; profiles/r01_vector_policy.txt).
template <int VP>
__device__ __forceinline__ d2 ldv(const double *p) {
    if constexpr (VP >= 2) return __builtin_nontemporal_load(reinterpret_cast<const d2 *>(p));
    else return *reinterpret_cast<const d2 *>(p);
}
template <int VP>
__device__ __forceinline__ void stv(double *p, d2 v) {
    if constexpr (VP >= 1) __builtin_nontemporal_store(v, reinterpret_cast<d2 *>(p));
    else *reinterpret_cast<d2 *>(p) = v;
}

// Vector kernels.  VEC (every pointer 16-B aligned): a block step covers
// kVU * kNT consecutive element pairs; each thread loads its kVU pairs of
// every input (16-B loads, all issued before any store), computes, stores.
// Otherwise a scalar grid-stride loop.  The odd tail element of the VEC
// path is done by thread 0 of block 0.  Per-thread sums run in a fixed
// order, then the deterministic grid reduction.
constexpr int kVU = 4;

#define CGX_VEC_LOOP_BEGIN                                                                   \
    const int64_t npairs = n >> 1;                                                           \
    const int64_t step = (int64_t)gridDim.x * kNT * kVU;                                     \
    for (int64_t base = (int64_t)blockIdx.x * kNT * kVU + threadIdx.x; base < npairs; base += step) { \
        bool ok[kVU];                                                                        \
        _Pragma("unroll") for (int u = 0; u < kVU; ++u) ok[u] = base + u * kNT < npairs;
#define CGX_VEC_LOOP_END }

// The device-side stopping decision of k_update_xp_f64 / k_poisson_p_f64
// (serialConjugate.c:235): eps < 0 disables it; kdone / rrfinal are device
// slots read by later launches' gates.
struct ConvArgs {
    double eps = -1.0;
    int64_t k = 0;
    int64_t *kdone = nullptr;   // 0 = not converged, else the loop-iteration count
    double *rrfinal = nullptr;
    int64_t *hrec = nullptr;    // host-mapped copy of {kdone, rrfinal}: read by the host without a copy
};

// The convergence record: device slots for later launches' gates, and the
// host-mapped copy the host reads after an event (no per-iteration D2H copy).
__device__ __forceinline__ void record_convergence(const ConvArgs &cv, int64_t kdone, double rr) {
    *cv.rrfinal = rr;
    *cv.kdone = kdone;
    if (cv.hrec) {
        __hip_atomic_store(cv.hrec + 1, __double_as_longlong(rr), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        __hip_atomic_store(cv.hrec, kdone, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    }
}

// ---------------------------------------------------------------------------
// counter-hash SPD generator (generateSPDmatrix.m:4-17 distribution)
// ---------------------------------------------------------------------------
__host__ __device__ __forceinline__ uint64_t mix64(uint64_t z) {
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}
__device__ __forceinline__ double u01(uint64_t salt, uint64_t i, uint64_t j) {
    const uint64_t h = mix64(((i << 32) | (j & 0xffffffffull)) ^ salt);
    return (double)(h >> 11) * 0x1.0p-53;
}

// ---------------------------------------------------------------------------
// host helpers
// ---------------------------------------------------------------------------
inline int cu_count(int device) {
    static std::mutex mu;
    static int cus[64] = {};
    std::lock_guard<std::mutex> lk(mu);
    if (device < 0 || device >= 64) return 256;
    if (cus[device] == 0) {
        int v = 0;
        if (hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, device) != hipSuccess || v <= 0)
            v = 256;
        cus[device] = v;
    }
    return cus[device];
}

inline int env_int(const char *name, int dflt) {
    const char *s = std::getenv(name);
    return (s && *s) ? std::atoi(s) : dflt;
}

// One key of a plan override held in one environment variable as
// "key=value,key=value" (CGX_MV_PLAN, CGX_SMALL_PLAN, CGX_POISSON_PLAN,
// CGX_SYM_PLAN): the value of `key`, or dflt.
inline int env_opt(const char *name, const char *key, int dflt) {
    const char *s = std::getenv(name);
    if (!s) return dflt;
    const size_t kl = std::strlen(key);
    for (const char *p = s; *p;) {
        if (std::strncmp(p, key, kl) == 0 && p[kl] == '=') return std::atoi(p + kl + 1);
        const char *q = std::strchr(p, ',');
        if (!q) break;
        p = q + 1;
    }
    return dflt;
}

inline unsigned grid_1d(int64_t n, int per_block, unsigned cap) {
    int64_t g = (n + per_block - 1) / per_block;
    if (g < 1) g = 1;
    if (g > (int64_t)cap) g = cap;
    return (unsigned)g;
}

// Grid of the vector kernels: <= kMaxRedBlocks (the partial slots), <= 8 blocks/CU.
inline unsigned grid_vec(int64_t n) { return grid_1d((n + 1) / 2, kNT * kVU, 2048); }

inline bool al16(const void *p) { return (reinterpret_cast<uintptr_t>(p) & 15) == 0; }

}  // namespace cgx
