// mrp_lane.h -- the lane kernels of one env id, included once per translation unit by
// mrp_env<E>.hip with MRP_ENV set (build.py compiles the seven units in parallel).
//
// Execution model: one wavefront (64 threads, one workgroup) owns one world ("lane").  The
// lane's persistent state is contiguous in HBM (lane-major, so the wave moves it with
// coalesced 16-B loads/stores) and lives in LDS for the whole step; order-sensitive Box2D
// work (tree updates, contact-list edits, events, island set-up) runs on thread 0, while
// the data-parallel phases (SAT narrow phase of every contact, broad-phase pair tests, TOI of
// every candidate contact, the island solver sweeps, state/obs I/O) are spread over the 64
// threads.  There is no dense contraction in this path, so no MFMA: the work is fp32 VALU with
// data-dependent control flow, plus fp64 for the env-level arithmetic.
#pragma once
#include <hip/hip_runtime.h>

#include <cstddef>
#include <cstring>
#include <type_traits>

#include "mrp_env.h"
#include "mrp_ops.h"
#include "../../include/mrp.h"

#ifndef MRP_ENV
#error "define MRP_ENV (the env id this translation unit instantiates)"
#endif
#ifdef MRP_STAMPS
static_assert(mrp::MRP_TRACE_W == MRP_TRACE_WORDS, "the trace row width is part of the C ABI (mrp_debug_trace)");
#endif

using namespace mrp;

// this unit's copy of its env's tables (uploaded by EnvOps::upload_tables at mrp_create)
static __constant__ EnvTables g_table;

#include "mrp_render.h"

namespace {
// LaneState is copied word-by-word; a may_alias word type keeps type-based alias analysis
// from reordering these copies against the typed (float/int) accesses of the step code.
typedef uint32_t __attribute__((__may_alias__)) word_t;

template <int ENV>
__device__ __forceinline__ void load_state(LaneState<ENV>& S, const uint32_t* __restrict__ g, int lane, int tid) {
    static_assert(sizeof(LaneState<ENV>) % 16 == 0, "lane state moves in 16-B granules");
    constexpr int NQ = (int)(sizeof(LaneState<ENV>) / 16);
    typedef uint4 __attribute__((__may_alias__)) quad_t;
    quad_t* w = reinterpret_cast<quad_t*>(&S);
    const quad_t* src = reinterpret_cast<const quad_t*>(g + (size_t)lane * lane_words<ENV>());
    for (int i = tid; i < NQ; i += BLOCK) w[i] = src[i];
}
template <int ENV>
__device__ __forceinline__ void store_state(const LaneState<ENV>& S, uint32_t* __restrict__ g, int lane, int tid) {
    constexpr int NQ = (int)(sizeof(LaneState<ENV>) / 16);
    typedef uint4 __attribute__((__may_alias__)) quad_t;
    const quad_t* w = reinterpret_cast<const quad_t*>(&S);
    quad_t* dst = reinterpret_cast<quad_t*>(g + (size_t)lane * lane_words<ENV>());
    for (int i = tid; i < NQ; i += BLOCK) dst[i] = w[i];
}

// words [A, B) of a lane's state, 16-B granules where aligned (A, B compile-time)
template <int A, int B, bool LOAD>
__device__ __forceinline__ void move_words(word_t* lds, word_t* g, int tid) {
    constexpr int QA = (A + 3) / 4, QB = B / 4;
    typedef uint4 __attribute__((__may_alias__)) quad_t;
    if (QA < QB) {
        for (int i = QA + tid; i < QB; i += BLOCK) {
            if (LOAD) reinterpret_cast<quad_t*>(lds)[i] = reinterpret_cast<const quad_t*>(g)[i];
            else reinterpret_cast<quad_t*>(g)[i] = reinterpret_cast<const quad_t*>(lds)[i];
        }
        constexpr int H = 4 * QA - A, T = B - 4 * QB;   // head / tail words outside the granules
        if (tid < H + T) {
            const int k = tid < H ? A + tid : 4 * QB + (tid - H);
            if (LOAD) lds[k] = g[k]; else g[k] = lds[k];
        }
    } else {
        for (int k = A + tid; k < B; k += BLOCK) { if (LOAD) lds[k] = g[k]; else g[k] = lds[k]; }
    }
}
// k_step's state round trip: everything but the contact slots >= cHW, which hold their initial
// contents in HBM and are rebuilt in LDS (LaneState::cHW).  `hw` = the slots to move (load: the
// stored cHW; store: max(cHW at load, cHW now), so slots a reset in this launch zeroed are
// written back as well).
//
// The load issues every global load of a region before its first wait (split issue / put), so a
// lane's state arrives in two memory round trips (the contact mark, then the live contact slots)
// instead of one per loop trip (~25 before) (round 4 A/B, profiles/r4_ab_batched_load_schedule.txt
// and r4_ab_contact_words.txt: v2 +2.9 %, the other configs +0-0.6 %).
typedef uint4 __attribute__((__may_alias__)) quad_t;
// words [A, B) of a lane's state: 16-B granules where aligned, single words at the ragged ends
template <int A, int B>
struct Span {
    static constexpr int QA = (A + 3) / 4, QB = B / 4;
    static constexpr bool QUADS = QA < QB;
    static constexpr int NQ = QUADS ? (QB - QA + BLOCK - 1) / BLOCK : 0;
    static constexpr int H = QUADS ? 4 * QA - A : 0, T = QUADS ? B - 4 * QB : 0;
    static constexpr int NS = QUADS ? 1 : (B - A + BLOCK - 1) / BLOCK;   // single words per thread
    quad_t q[NQ > 0 ? NQ : 1];
    word_t s[NS > 0 ? NS : 1];
    __device__ __forceinline__ static int single(int tid, int k) {
        if constexpr (QUADS) return tid < H ? A + tid : 4 * QB + (tid - H);
        else return A + tid + k * BLOCK;
    }
    __device__ __forceinline__ static bool has_single(int tid, int k) {
        if constexpr (QUADS) return tid < H + T;
        else return A + tid + k * BLOCK < B;
    }
    __device__ __forceinline__ void issue(const word_t* g, int tid) {
#pragma unroll
        for (int k = 0; k < NQ; ++k) {
            const int i = QA + tid + k * BLOCK;
            if (i < QB) q[k] = reinterpret_cast<const quad_t*>(g)[i];
        }
#pragma unroll
        for (int k = 0; k < NS; ++k)
            if (has_single(tid, k)) s[k] = g[single(tid, k)];
    }
    __device__ __forceinline__ void put(word_t* lds, int tid) const {
#pragma unroll
        for (int k = 0; k < NQ; ++k) {
            const int i = QA + tid + k * BLOCK;
            if (i < QB) reinterpret_cast<quad_t*>(lds)[i] = q[k];
        }
#pragma unroll
        for (int k = 0; k < NS; ++k)
            if (has_single(tid, k)) lds[single(tid, k)] = s[k];
    }
};
template <int ENV>
struct StateIO {
    using LS = LaneState<ENV>;
    static constexpr int C = LS::C;
    static constexpr int P = (int)(offsetof(LS, cnext) / 4), Q = (int)(offsetof(LS, inv_dt0) / 4), NW = lane_words<ENV>();
    static constexpr int HWW = (int)(offsetof(LS, cHW) / 4);
    static_assert(Q - P == LS::NCA * C, "contact arrays cnext .. mid[1] are contiguous");
    // The contact slots' words [P, Q): NCA arrays of C words, slot c of array a at word
    // P + a * C + c; only slots below the mark hw are live and move, word by word (ContactWords) or
    // in 16-B granules (ContactGranules, MRP_CONTACT_GRANULES=1: the v2 unit, +2.5 % there; for v0
    // and v3 level in time and +16 % in PMC traffic, profiles/r4_ab_contact_granules.txt).
    // The load issues every live word's load before the first wait and puts the initial contents
    // into the other words.
    struct ContactWords {
        static constexpr int NWC = LS::NCA * C, NK = (NWC + BLOCK - 1) / BLOCK;
        word_t w[NK];
        __device__ __forceinline__ static bool live(int i, int hw) { return i % C < hw; }   // i: word of the region
        __device__ __forceinline__ static word_t init(int i) {
            // cnext (array 0) chains the free list 0 -> 1 -> ... -> C-1; the other arrays are 0
            return i < C ? (i + 1 < C ? (word_t)(i + 1) : (word_t)NULLN) : 0u;
        }
        __device__ __forceinline__ void issue(const word_t* g, int hw, int tid) {
#pragma unroll
            for (int k = 0; k < NK; ++k) {
                const int i = tid + k * BLOCK;
                if ((i < NWC) & live(i, hw)) w[k] = g[P + i];
            }
        }
        __device__ __forceinline__ void put(word_t* lds, int hw, int tid) const {
#pragma unroll
            for (int k = 0; k < NK; ++k) {
                const int i = tid + k * BLOCK;
                if (i < NWC) lds[P + i] = live(i, hw) ? w[k] : init(i);
            }
        }
        __device__ __forceinline__ static void store(const word_t* lds, word_t* g, int hw, int tid) {
#pragma unroll
            for (int k = 0; k < NK; ++k) {
                const int i = tid + k * BLOCK;
                if ((i < NWC) & live(i, hw)) g[P + i] = lds[P + i];
            }
        }
    };
    // The same words moved in 16-B granules: a granule with any live word moves whole; its other
    // words hold their initial contents on both sides (in HBM by the cHW invariant, in LDS because
    // the load puts them there and the step takes slots only at the mark), and the load replaces
    // them by those contents word by word (MRP_CONTACT_GRANULES=1: fewer, wider loads, more traffic)
    struct ContactGranules {
        static constexpr int QA = (P + 3) / 4, QB = Q / 4, NQ = (QB - QA + BLOCK - 1) / BLOCK;
        static constexpr int H = 4 * QA - P, T = Q - 4 * QB;
        static_assert(QA < QB && H + T < BLOCK, "contact words span whole granules");
        quad_t q[NQ];
        word_t s;
        __device__ __forceinline__ static bool live(int w, int hw) { return (w - P) % C < hw; }
        __device__ __forceinline__ static word_t init(int w) {
            const int i = w - P;   // cnext (array 0) chains the free list 0 -> 1 -> ... -> C-1; the rest are 0
            return i < C ? (i + 1 < C ? (word_t)(i + 1) : (word_t)NULLN) : 0u;
        }
        // granule j's first slot; its words are slots c0 .. c0 + 3, wrapping into the next array's
        // slots 0, 1, 2 (C >= 4), so it is live iff c0 < hw or it wraps and slot 0 is live
        __device__ __forceinline__ static int slot0(int j) { return (4 * j - P) % C; }
        __device__ __forceinline__ static bool quad_live(int c0, int hw) { return (c0 < hw) | ((c0 + 3 >= C) & (hw > 0)); }
        __device__ __forceinline__ static word_t pick(word_t v, int c, int w, int hw) {
            return (c >= C ? c - C : c) < hw ? v : init(w);
        }
        static_assert(C >= 4, "a granule spans at most two arrays");
        __device__ __forceinline__ static int single(int tid) { return tid < H ? P + tid : 4 * QB + (tid - H); }
        __device__ __forceinline__ void issue(const word_t* g, int hw, int tid) {
#pragma unroll
            for (int k = 0; k < NQ; ++k) {
                const int j = QA + tid + k * BLOCK;
                if ((j < QB) & quad_live(slot0(j), hw)) q[k] = reinterpret_cast<const quad_t*>(g)[j];
            }
            if ((tid < H + T) & live(single(tid), hw)) s = g[single(tid)];
        }
        __device__ __forceinline__ void put(word_t* lds, int hw, int tid) const {
#pragma unroll
            for (int k = 0; k < NQ; ++k) {
                const int j = QA + tid + k * BLOCK;
                if (j < QB) {
                    const int c0 = slot0(j);
                    quad_t v = q[k];
                    v.x = pick(v.x, c0, 4 * j, hw);
                    v.y = pick(v.y, c0 + 1, 4 * j + 1, hw);
                    v.z = pick(v.z, c0 + 2, 4 * j + 2, hw);
                    v.w = pick(v.w, c0 + 3, 4 * j + 3, hw);
                    reinterpret_cast<quad_t*>(lds)[j] = v;
                }
            }
            if (tid < H + T) lds[single(tid)] = live(single(tid), hw) ? s : init(single(tid));
        }
        __device__ __forceinline__ static void store(const word_t* lds, word_t* g, int hw, int tid) {
#pragma unroll
            for (int k = 0; k < NQ; ++k) {
                const int j = QA + tid + k * BLOCK;
                if ((j < QB) & quad_live(slot0(j), hw)) reinterpret_cast<quad_t*>(g)[j] = reinterpret_cast<const quad_t*>(lds)[j];
            }
            if ((tid < H + T) & live(single(tid), hw)) g[single(tid)] = lds[single(tid)];
        }
    };
#ifndef MRP_CONTACT_GRANULES
#define MRP_CONTACT_GRANULES 0
#endif
#ifndef MRP_FRESH_REGS
#define MRP_FRESH_REGS 0
#endif
    using Contacts = typename std::conditional<MRP_CONTACT_GRANULES != 0, ContactGranules, ContactWords>::type;
    // hw_io <- the loaded cHW (clamped to the pool; kept in LDS, not live in registers across the step)
    __device__ __forceinline__ static void load(LS& S, int& hw_io, const uint32_t* __restrict__ gs, int lane, int tid) {
        const word_t* g = gs + (size_t)lane * NW;
        word_t* lds = reinterpret_cast<word_t*>(&S);
        const word_t mark = g[HWW];
        Span<0, P> head;
        Span<Q, NW> tail;
        head.issue(g, tid);
        tail.issue(g, tid);
        const int hw = min(max((int)__builtin_amdgcn_readfirstlane(mark), 0), C);
        Contacts ct;
        ct.issue(g, hw, tid);
        head.put(lds, tid);
        tail.put(lds, tid);
        ct.put(lds, hw, tid);
        if (tid == 0) hw_io = hw;
    }
    __device__ __forceinline__ static void store(const LS& S, const int& hw_io, uint32_t* __restrict__ gs, int lane, int tid) {
#if MRP_FRESH_REGS
        // the per-thread word offsets recomputed here from an opaque copy of the thread id, not kept
        // live from the load at entry (v0 under the iterative-ilp schedule spilled two of them to
        // scratch across the whole step)
        asm volatile("" : "+v"(tid));
#endif
        word_t* g = gs + (size_t)lane * NW;
        word_t* lds = const_cast<word_t*>(reinterpret_cast<const word_t*>(&S));
        const int hw = max(hw_io, min(max(S.cHW, 0), C));
        move_words<0, P, false>(lds, g, tid);
        move_words<Q, NW, false>(lds, g, tid);
        Contacts::store(lds, g, hw, tid);
    }
};

// copy this env's hot tables from __constant__ memory into the lane's LDS (before the
// barrier that follows load_state)
template <int ENV>
__device__ __forceinline__ void load_tables(LdsTables<ENV>& L, int tid) {
    using LT = LdsTables<ENV>;
    const EnvTables& T = g_table;
    constexpr int SW = LT::NF * (int)(sizeof(ShapeDef) / 4);
    const word_t* src = reinterpret_cast<const word_t*>(T.shape);
    word_t* dst = reinterpret_cast<word_t*>(L.shape);
    for (int i = tid; i < SW; i += BLOCK) dst[i] = src[i];
    if (tid < LT::NF) {
        L.fix_body[tid] = T.fix_body[tid]; L.fix_friction[tid] = T.fix_friction[tid];
        L.fix_restitution[tid] = T.fix_restitution[tid];
    }
    if (tid < LT::NBODY) {
        L.invMass[tid] = T.invMass[tid]; L.invI[tid] = T.invI[tid]; L.lcx[tid] = T.lcx[tid]; L.lcy[tid] = T.lcy[tid];
        L.linDamp[tid] = T.linDamp[tid]; L.angDamp[tid] = T.angDamp[tid];
        L.body_fix0[tid] = T.body_fix0[tid]; L.body_nfix[tid] = T.body_nfix[tid];
    }
    if (tid < 4) { L.wall_px[tid] = T.wall_px[tid]; L.wall_py[tid] = T.wall_py[tid]; }
}

template <int ENV>
__global__ __launch_bounds__(BLOCK) void k_init(uint32_t* state, int nl) {
    __shared__ Shared<ENV> sh;
    const int lane = blockIdx.x, tid = threadIdx.x;
    if (lane >= nl) return;
    word_t* w = reinterpret_cast<word_t*>(&sh.S);
    for (int i = tid; i < lane_words<ENV>(); i += BLOCK) w[i] = 0;
    __syncthreads();
    if (tid == 0) {
        EnvParams P;
        memset(&P, 0, sizeof(P));
        Env<ENV> e(sh, g_table, P, 0);
        e.init_empty_world();
    }
    __syncthreads();
    store_state<ENV>(sh.S, state, lane, tid);
}

// stage one reset's draws/action into LDS: host-provided rows or the counter RNG
template <int ENV>
__device__ void stage_reset_inputs(Shared<ENV>& sh, const double* draws, const float* actions, int lane, int tid,
                                   uint64_t seed, uint64_t glane) {
    using D = Dims<ENV>;
    const EnvTables& T = g_table;
    const uint64_t ctr = (uint64_t)(uint32_t)sh.S.episode * 64u;
    if (tid < D::NDRAW)
        sh.draws[tid] = draws ? draws[(size_t)lane * D::NDRAW + tid]
                              : T.draw_lo[tid] + (T.draw_hi[tid] - T.draw_lo[tid]) * rng_u01(seed, glane, 1, ctr + tid);
    if (tid < D::ACT)
        sh.act[tid] = actions ? actions[(size_t)lane * D::ACT + tid] : (float)(-1.0 + 2.0 * rng_u01(seed, glane, 2, ctr + tid));
    __syncthreads();
    if (tid == 0) { sh.S.episode += 1; sh.S.elapsed = 0; }
    __syncthreads();
}

template <int ENV>
__global__ __launch_bounds__(BLOCK, 4) void k_reset(uint32_t* state, int nl, const uint8_t* mask, const double* draws,
                                                 const float* actions, float* obs, EnvParams P, uint64_t seed,
                                                 uint64_t lane_offset) {
    using D = Dims<ENV>;
    __shared__ Shared<ENV> sh;
    const int lane = blockIdx.x, tid = threadIdx.x;
    if (lane >= nl) return;
    if (mask && !mask[lane]) return;
    load_state<ENV>(sh.S, state, lane, tid);
    load_tables<ENV>(sh.lt, tid);
    __syncthreads();
    stage_reset_inputs<ENV>(sh, draws, actions, lane, tid, seed, lane_offset + lane);
    Env<ENV> e(sh, g_table, P, tid);
    e.env_reset_coop();
    for (int k = tid; k < D::OBS; k += BLOCK) obs[(size_t)lane * D::OBS + k] = sh.obs[k];
    store_state<ENV>(sh.S, state, lane, tid);
}

template <int ENV, bool MULTI>
#ifndef MRP_STEP_WAVES_PER_EU
// 3 waves per SIMD (168 VGPRs): k_step without VGPR spills in the solver phases.  At 4 (128 VGPRs,
// all 4096 lanes of a GPU resident at once) the kernel carried 54 VGPR spills whose scratch traffic
// was 12.7 MB of its 46.7 MB per v0 launch; the driver window runs at the same rate either way
// (profiles/r3c_ab_occ3_regs3.txt, profiles/r3c_ab_occ3_trim.txt, profiles/r3c_traffic_occ3_trim.txt)
#define MRP_STEP_WAVES_PER_EU 3
#endif
__global__ __launch_bounds__(BLOCK, MRP_STEP_WAVES_PER_EU) void k_step(uint32_t* state, int nl, const float* actions, float* obs, float* reward,
                                                double* reward64, uint8_t* done_out, uint8_t* trunc_out, uint8_t* status_out, float* term_obs,
                                                EnvParams P, uint64_t seed, uint64_t lane_offset, int auto_reset,
                                                int max_steps, const int* __restrict__ order, uint32_t* __restrict__ cost,
                                                const uint32_t* __restrict__ costmax, int nsteps) {
    using D = Dims<ENV>;
    __shared__ Shared<ENV> sh;
    __shared__ int s_fin;
    const int tid = threadIdx.x;
    if ((int)blockIdx.x >= nl) return;
    // workgroup b steps lane order[b]: the previous step's costliest lanes are dispatched first
    // (k_order), so no SIMD collects several long serial chains; a lane's result does not depend
    // on which workgroup steps it
    const int lane = order ? order[blockIdx.x] : (int)blockIdx.x;
    const unsigned long long t_start = cost ? __builtin_amdgcn_s_memtime() : 0ull;
    const uint64_t glane = lane_offset + lane;
#ifdef MRP_STAMPS
    if (tid == 0) { sh.stamp_t = sh.stamp_t0 = __builtin_amdgcn_s_memtime(); sh.stamp_rt0 = __builtin_amdgcn_s_memrealtime(); }
    if (tid < MRP_TRACE_W) sh.trace[tid] = 0;
    long long toi0 = 0, pos0 = 0;
#endif
    StateIO<ENV>::load(sh.S, sh.hw_io, state, lane, tid);
#ifdef MRP_STAMPS
    if (tid == 0) sh.trace[24] = (uint32_t)(__builtin_amdgcn_s_memtime() - sh.stamp_t0);
#endif
    load_tables<ENV>(sh.lt, tid);
#ifdef MRP_STAMPS
    if (tid == 0) sh.trace[25] = (uint32_t)(__builtin_amdgcn_s_memtime() - sh.stamp_t0);
#endif
    __syncthreads();
#ifdef MRP_STAMPS
    toi0 = sh.S.toiEvents; pos0 = sh.S.posIters;
    if (tid == 0) sh.trace[26] = (uint32_t)(__builtin_amdgcn_s_memtime() - sh.stamp_t0);
#endif
    MRP_STAMP(0);
    Env<ENV> e(sh, g_table, P, tid);
    if (costmax) {   // priority from the lane's previous-step cost relative to the slowest lane's
        const uint64_t c = cost[lane], m = *costmax;
        e.prio_floor = __builtin_amdgcn_readfirstlane(4 * c > 3 * m ? 3 : (2 * c > m ? 2 : (4 * c > m ? 1 : 0)));
        e.set_prio(e.prio_floor);
    }
    // nsteps > 1 (mrp_step_n_device): the lane advances nsteps env steps with its state resident in
    // LDS, writing every step's outputs (row s * nl + lane); each step is exactly one mrp_step
    // (the single-step instantiation has a compile-time trip count of one, so none of the loop's
    // state stays live across steps: the multi-step form carries more registers)
    const int ns = MULTI ? nsteps : 1;
    for (int s = 0; s < ns; ++s) {
        const size_t row = (size_t)s * nl + lane;
        const uint64_t ctr = (uint64_t)sh.S.stepCounter * 64u;
        if (tid < D::ACT)
            sh.act[tid] = actions ? actions[row * D::ACT + tid] : (float)(-1.0 + 2.0 * rng_u01(seed, glane, 3, ctr + tid));
        __syncthreads();
        if (tid == 0) sh.S.stepCounter += 1;
        e.env_step_coop();
        // per-lane failure report (SURVEY.md 8b Errors): a NaN / inf in the observation or the
        // dynamic bodies' state, and a sticky loop-guard fault, set status bits (never a crash)
        bool nf = false;
        for (int k = tid; k < D::OBS; k += BLOCK) nf |= !__builtin_isfinite(sh.obs[k]);
        if (tid < LaneState<ENV>::ND) {
            const int b = tid;
            nf |= !__builtin_isfinite(sh.S.cx[b]) || !__builtin_isfinite(sh.S.cy[b]) || !__builtin_isfinite(sh.S.a[b]) ||
                  !__builtin_isfinite(sh.S.vx[b]) || !__builtin_isfinite(sh.S.vy[b]) || !__builtin_isfinite(sh.S.w[b]);
        }
        const bool nonfinite = __builtin_amdgcn_ballot_w64(nf) != 0;
        if (tid == 0) {
            sh.S.elapsed += 1;
            int d = sh.done, tr = 0;
            if (max_steps > 0 && sh.S.elapsed >= max_steps) { tr = !d; d = 1; }   // gym TimeLimit
            if (nonfinite) sh.S.nonfinite += 1;
            if (reward) reward[row] = (float)sh.reward;
            if (reward64) reward64[row] = sh.reward;   // the reference's Python float
            if (done_out) done_out[row] = (uint8_t)d;
            if (trunc_out) trunc_out[row] = (uint8_t)tr;
            if (status_out)
                status_out[row] = (uint8_t)(sh.kind | (nonfinite ? MRP_STATUS_NONFINITE_BIT : 0) |
                                            (sh.S.fault ? MRP_STATUS_FAULT_BIT : 0));
            s_fin = d;
        }
        __syncthreads();
        if (term_obs)
            for (int k = tid; k < D::OBS; k += BLOCK) term_obs[row * D::OBS + k] = sh.obs[k];
        MRP_STAMP(8);
        if (s_fin && auto_reset) {   // SB3-style auto-reset with device-RNG spawns
            stage_reset_inputs<ENV>(sh, nullptr, nullptr, lane, tid, seed, glane);
            e.env_reset_coop();
            MRP_STAMP(9);
        }
        for (int k = tid; k < D::OBS; k += BLOCK) obs[row * D::OBS + k] = sh.obs[k];
        __syncthreads();
    }
    StateIO<ENV>::store(sh.S, sh.hw_io, state, lane, tid);
    if (cost && tid == 0) cost[lane] = (uint32_t)min(__builtin_amdgcn_s_memtime() - t_start, 0xffffffffull);
    MRP_STAMP(10);
#ifdef MRP_STAMPS
    // no global atomics here: the totals are folded from the traces by k_stamp_fold after the
    // launch (up to round 4 this block issued 25 atomics per lane on the same few words, and
    // the other lanes' loads and stores queued behind them at the L2)
    if (tid == 0) {
        unsigned long long tot = sh.stamp_t - sh.stamp_t0;
        sh.trace[11] = (uint32_t)tot;
        sh.trace[27] = (sh.S.stepCounter - 1u) & 255u;
        sh.trace[13] = (uint32_t)(sh.S.toiEvents - toi0);
        sh.trace[14] = (uint32_t)(sh.S.posIters - pos0);
        // where and when the lane ran: s_memrealtime (100 MHz, chip-wide) at entry and at the end,
        // HW_ID (wave / SIMD / CU / SE) and XCC_ID, so a launch's last lane can be named
        sh.trace[28] = (uint32_t)sh.stamp_rt0;
        sh.trace[29] = (uint32_t)__builtin_amdgcn_s_memrealtime();
        sh.trace[30] = (uint32_t)__builtin_amdgcn_s_getreg((31 << 11) | 4);
        sh.trace[31] = (uint32_t)__builtin_amdgcn_s_getreg((31 << 11) | 20);
    }
    __syncthreads();
    if (tid < MRP_TRACE_W && lane < 16384) g_trace[lane][tid] = sh.trace[tid];
#endif
}

#ifdef MRP_STAMPS
// diagnostic builds: folds one launch's per-lane traces into the stamp totals read by
// mrp_debug_stamps / mrp_debug_stamps_ext (phase sums and maxima, lane-total sums in s_memtime
// and s_memrealtime ticks, the slowest lane per step), one workgroup after k_step
template <int ENV>
__global__ __launch_bounds__(256) void k_stamp_fold(int nl) {
    constexpr int R = 25;   // 0-10 phase sums, 11-21 phase maxima, 22/23 total sums, 24 slowest lane of the common step
    __shared__ unsigned long long red[R][256];
    const int t = threadIdx.x, n = nl < 16384 ? nl : 16384;
    unsigned long long acc[R] = {};
    const uint32_t step0 = n > 0 ? (g_trace[0][27] & 255u) : 0u;
    for (int l = t; l < n; l += 256) {
        const uint32_t* w = g_trace[l];
        for (int k = 0; k < 11; ++k) { acc[k] += w[k]; acc[11 + k] = acc[11 + k] > w[k] ? acc[11 + k] : w[k]; }
        acc[22] += w[11];
        acc[23] += (uint32_t)(w[29] - w[28]);
        if ((w[27] & 255u) == step0) acc[24] = acc[24] > w[11] ? acc[24] : w[11];
        else atomicMax(&g_stepmax[w[27] & 255u], (unsigned long long)w[11]);   // lanes reset on another step
    }
    for (int k = 0; k < R; ++k) red[k][t] = acc[k];
    __syncthreads();
    for (int h = 128; h > 0; h >>= 1) {
        if (t < h)
            for (int k = 0; k < R; ++k) {
                const unsigned long long a = red[k][t], b = red[k][t + h];
                red[k][t] = (k >= 11 && k < 22) || k == 24 ? (a > b ? a : b) : a + b;
            }
        __syncthreads();
    }
    if (t == 0) {
        for (int k = 0; k < 11; ++k) { atomicAdd(&g_stamps[k], red[k][0]); atomicMax(&g_pmax[k], red[11 + k][0]); }
        atomicAdd(&g_rt[0], red[22][0]);
        atomicAdd(&g_rt[1], red[23][0]);
        atomicMax(&g_stepmax[step0], red[24][0]);
    }
}
#endif

template <int ENV>
__global__ __launch_bounds__(BLOCK) void k_bodies(const uint32_t* state, int nl, float* out, int32_t* flags) {
    using D = Dims<ENV>;
    const int lane = blockIdx.x, tid = threadIdx.x;
    if (lane >= nl || tid != 0) return;
    const LaneState<ENV>& S = *reinterpret_cast<const LaneState<ENV>*>(state + (size_t)lane * lane_words<ENV>());
    constexpr int ND = D::NA + D::NB;
    if (out) {
        float* r = out + (size_t)lane * 6 * ND;
        for (int b = 0; b < ND; ++b) {
            r[6 * b] = S.cx[b]; r[6 * b + 1] = S.cy[b]; r[6 * b + 2] = S.a[b];
            r[6 * b + 3] = S.vx[b]; r[6 * b + 4] = S.vy[b]; r[6 * b + 5] = S.w[b];
        }
    }
    if (flags) {
        int32_t* f = flags + (size_t)lane * (D::NA + 1);
        for (int i = 0; i < D::NA; ++i) f[i] = S.goal_contact[i];
        f[D::NA] = S.blks_in_place;
    }
}

template <int ENV>
__global__ __launch_bounds__(256) void k_faults(const uint32_t* state, int nl, int32_t* out) {
    const int lane = blockIdx.x * 256 + threadIdx.x;
    if (lane >= nl) return;
    const LaneState<ENV>& S = *reinterpret_cast<const LaneState<ENV>*>(state + (size_t)lane * lane_words<ENV>());
    out[lane] = S.fault;
}

// per-lane counters summed over the lanes (one workgroup; a tree reduction in LDS, no atomics)
template <int ENV>
__global__ __launch_bounds__(256) void k_counters(const uint32_t* state, int nl, int64_t* out) {
    __shared__ long long red[CTR_N][256];
    const int t = threadIdx.x;
    long long acc[CTR_N] = {};
    for (int lane = t; lane < nl; lane += 256) {
        const LaneState<ENV>& S = *reinterpret_cast<const LaneState<ENV>*>(state + (size_t)lane * lane_words<ENV>());
        acc[CTR_STEPS] += S.stepCounter; acc[CTR_RESETS] += S.episode; acc[CTR_TOI] += S.toiEvents;
        acc[CTR_POS_ITERS] += S.posIters; acc[CTR_TOUCHING] += S.touching; acc[CTR_NONFINITE] += S.nonfinite;
        acc[CTR_FAULT_LANES] += S.fault != 0;
    }
    for (int k = 0; k < CTR_N; ++k) red[k][t] = acc[k];
    __syncthreads();
    for (int w = 128; w > 0; w >>= 1) {
        if (t < w)
            for (int k = 0; k < CTR_N; ++k) red[k][t] += red[k][t + w];
        __syncthreads();
    }
    if (t < CTR_N) out[t] = red[t][0];
}

// ------------------------------------------------------------------------------ launch table
template <int ENV>
struct Launch {
    static hipError_t upload_tables(const EnvTables* all) {
        return hipMemcpyToSymbol(HIP_SYMBOL(g_table), all + ENV, sizeof(EnvTables));
    }
    static void init(hipStream_t s, uint32_t* state, int nl) {
        hipLaunchKernelGGL(k_init<ENV>, dim3(nl), dim3(BLOCK), 0, s, state, nl);
    }
    static void reset(hipStream_t s, uint32_t* state, int nl, const uint8_t* mask, const double* draws, const float* actions,
                      float* obs, const EnvParams& P, uint64_t seed, uint64_t lane_offset) {
        hipLaunchKernelGGL(k_reset<ENV>, dim3(nl), dim3(BLOCK), 0, s, state, nl, mask, draws, actions, obs, P, seed, lane_offset);
    }
    static void step(hipStream_t s, const StepArgs& a) {
        if (a.nsteps > 1)
            hipLaunchKernelGGL((k_step<ENV, true>), dim3(a.nl), dim3(BLOCK), 0, s, a.state, a.nl, a.actions, a.obs, a.reward,
                               a.reward64, a.done, a.trunc, a.status, a.term_obs, a.P, a.seed, a.lane_offset, a.auto_reset,
                               a.max_steps, a.order, a.cost, a.costmax, a.nsteps);
        else
            hipLaunchKernelGGL((k_step<ENV, false>), dim3(a.nl), dim3(BLOCK), 0, s, a.state, a.nl, a.actions, a.obs, a.reward,
                               a.reward64, a.done, a.trunc, a.status, a.term_obs, a.P, a.seed, a.lane_offset, a.auto_reset,
                               a.max_steps, a.order, a.cost, a.costmax, 1);
#ifdef MRP_STAMPS
        hipLaunchKernelGGL(k_stamp_fold<ENV>, dim3(1), dim3(256), 0, s, a.nl);
#endif
    }
    static void bodies(hipStream_t s, const uint32_t* state, int nl, float* out, int32_t* flags) {
        hipLaunchKernelGGL(k_bodies<ENV>, dim3(nl), dim3(BLOCK), 0, s, state, nl, out, flags);
    }
    static void faults(hipStream_t s, const uint32_t* state, int nl, int32_t* out) {
        hipLaunchKernelGGL(k_faults<ENV>, dim3((nl + 255) / 256), dim3(256), 0, s, state, nl, out);
    }
    static void counters(hipStream_t s, const uint32_t* state, int nl, int64_t* out) {
        hipLaunchKernelGGL(k_counters<ENV>, dim3(1), dim3(256), 0, s, state, nl, out);
    }
    static void render(hipStream_t s, dim3 grid, const uint32_t* state, const int32_t* lanes, int nl, int W, int H,
                       const mrpr::RenderArgs& A, uint8_t* rgb) {
        hipLaunchKernelGGL(mrpr::k_render<ENV>, grid, dim3(mrpr::RBLOCK), 0, s, state, lanes, nl, W, H, A, rgb);
    }
    static void goals(hipStream_t s, const uint32_t* state, int nl, double* out) {
        hipLaunchKernelGGL(mrpr::k_goals<ENV>, dim3((nl + 255) / 256), dim3(256), 0, s, state, nl, out);
    }
    static hipError_t debug_read(int what, void* out, size_t bytes) {
#ifdef MRP_STAMPS
        static char zero[16384 * 16 * 4];
        hipError_t e = hipDeviceSynchronize();
        const void* sym = what == DBG_STAMPS ? (const void*)HIP_SYMBOL(g_stamps) : what == DBG_PMAX ? (const void*)HIP_SYMBOL(g_pmax)
                        : what == DBG_STEPMAX ? (const void*)HIP_SYMBOL(g_stepmax) : what == DBG_RT ? (const void*)HIP_SYMBOL(g_rt)
                        : (const void*)HIP_SYMBOL(g_trace);
        if (e == hipSuccess) e = hipMemcpyFromSymbol(out, sym, bytes);
        if (e == hipSuccess && what != DBG_TRACE) e = hipMemcpyToSymbol(sym, zero, bytes);
        return e;
#else
        (void)what; (void)out; (void)bytes;
        return hipErrorNotSupported;
#endif
    }
    static hipError_t debug_progress(uint32_t* dev_words) {
#ifdef MRP_PROGRESS
        return hipMemcpyToSymbol(HIP_SYMBOL(g_progress), &dev_words, sizeof(dev_words));
#else
        (void)dev_words;
        return hipErrorNotSupported;
#endif
    }
    static constexpr EnvOps ops() {
        using D = Dims<ENV>;
        using LS = LaneState<ENV>;
        return EnvOps{lane_words<ENV>(), (int)(offsetof(LS, toiEvents) / 4),
                      {D::OBS, D::ACT, D::NDRAW, D::NA, D::NB, D::NF},
                      StateIO<ENV>::P, LS::C, LS::NCA, StateIO<ENV>::HWW, MRP_STEP_WAVES_PER_EU, upload_tables, init, reset, step,
                      bodies, faults, counters, render, goals, debug_read, debug_progress};
    }
};

}  // namespace

// the table is host data: the device-side pass of the unit must not see its initializer, but
// it must instantiate the kernels the launchers name
#if defined(__HIP_DEVICE_COMPILE__)
#define MRP_DEFINE_ENV_OPS(E) namespace { template struct Launch<E>; }
#else
#define MRP_DEFINE_ENV_OPS(E) \
    namespace mrp { extern const EnvOps g_env_ops_##E; const EnvOps g_env_ops_##E = Launch<E>::ops(); }
#endif

#if MRP_ENV == 0
namespace {
// Diagnostic micro-benchmark of the lane-distributed velocity sweeps (mrp_debug_velbench): a
// synthetic v0 island of nc agent-block contacts with pcount manifold points each, swept `iters`
// times with the early exit off; out[block] = s_memtime cycles of the sweeps.
__global__ __launch_bounds__(BLOCK, MRP_STEP_WAVES_PER_EU) void k_velbench(int nc, int pcount, int iters, unsigned long long* out) {
    using W = World<0>;
    __shared__ Shared<0> sh;
    const int tid = threadIdx.x;
    EnvParams P{};
    W w(sh, g_table, P, tid);
    auto& is = sh.isl;
    // nc >= 100: a chain of nc - 100 contacts (contact i between bodies i and i + 1, all moving)
    const bool chain = nc >= 100;
    if (chain) nc -= 100;
    if (tid == 0) {
        is.nb = nc + 1; is.nc = nc;
        for (int b = 0; b <= nc; ++b) { is.vvx[b] = 0.3f * b - 0.1f; is.vvy[b] = 0.2f - 0.05f * b; is.vw[b] = b == 0 ? 0.01f : 0.0f; }
        for (int i = 0; i < nc; ++i) {
            VC& vc = sh.u.sol.vcs[i];
            const float ang = 0.7f * (float)i + 0.3f;
            vc.nx = __cosf(ang); vc.ny = __sinf(ang);
            vc.iaI = i + 1; vc.ibI = 0; vc.mA = 1.0f; vc.iA = 0.0f; vc.mB = 0.05f; vc.iB = 1.0f / 17.0833f; vc.friction = 0.44f;
            vc.pointCount = pcount;
            if (chain) { vc.iaI = i; vc.ibI = i + 1; vc.mA = 1.0f; vc.iA = 0.05f; }
            for (int j = 0; j < 2; ++j) {
                vc.rAx[j] = 0.1f * j - 0.2f; vc.rAy[j] = 0.75f; vc.rBx[j] = 0.4f + 0.3f * j; vc.rBy[j] = -0.6f;
                vc.ni[j] = 0.2f; vc.ti[j] = 0.01f; vc.vbias[j] = 0.0f; vc.nmass[j] = 0.9f; vc.tmass[j] = 0.8f;
            }
            vc.k0 = 1.2f; vc.k1 = 0.3f; vc.k3 = 1.1f; vc.nm0 = 0.9f; vc.nm1 = -0.2f; vc.nm3 = 0.95f;
        }
    }
    __syncthreads();
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    int sw = nc == 1 ? w.solver_velocity_one(is, sh.u.sol.vcs, iters, false)
                     : (nc == 2 ? w.solver_velocity_two(is, sh.u.sol.vcs, iters, false) : -1);
    if (sw < 0) w.solver_velocity_lanes(is, sh.u.sol.vcs, iters, false);
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    __syncthreads();
    if (tid == 0) out[blockIdx.x] = t1 - t0 + (is.vvx[0] == 12345.0f ? 1ull : 0ull);
}
// Diagnostic micro-benchmark of the position passes (mrp_debug_posbench): a synthetic island of nc
// static-wall contacts of pcount points on one moving block (body 0), walls alternately above and
// below it, each penetrating it by ~0.1 (the squeezed shape of the slowest v0 lanes: the passes never
// reach the exit test), solved by the dispatch of the step (register paths for 1-2 contacts, the
// lanes path above); out[2 * block] = s_memtime cycles, out[2 * block + 1] = passes run.
__global__ __launch_bounds__(BLOCK, MRP_STEP_WAVES_PER_EU) void k_posbench(int nc, int pcount, int iters, unsigned long long* out) {
    using W = World<0>;
    __shared__ Shared<0> sh;
    const int tid = threadIdx.x;
    EnvParams P{};
    W w(sh, g_table, P, tid);
    auto& is = sh.isl;
    if (tid == 0) {
        is.nb = nc + 1; is.nc = nc;
        is.pcx[0] = 0.0f; is.pcy[0] = 0.0f; is.pa[0] = 0.3f; is.vvx[0] = 0.0f; is.vvy[0] = 0.0f; is.vw[0] = 0.0f;
        for (int i = 0; i < nc; ++i) {
            const float up = (i & 1) ? -1.0f : 1.0f;   // wall above (normal down) or below (normal up)
            is.pcx[i + 1] = 0.05f * (float)i; is.pcy[i + 1] = up; is.pa[i + 1] = 0.0f;
            is.vvx[i + 1] = 0.0f; is.vvy[i + 1] = 0.0f; is.vw[i + 1] = 0.0f;
            VC& vc = sh.u.sol.vcs[i];
            PC& pc = sh.u.sol.pcs[i];
            vc.iaI = i + 1; vc.ibI = 0; vc.mA = 0.0f; vc.iA = 0.0f; vc.mB = 0.05f; vc.iB = 1.0f / 17.0833f;
            vc.pointCount = pcount;
            pc.type = MT_FACEA; pc.pointCount = pcount;
            pc.lnx = 0.0f; pc.lny = -up; pc.lpx0 = 0.0f; pc.lpy0 = -0.5f * up;
            pc.lpx[0] = -0.2f; pc.lpy[0] = 0.62f * up; pc.lpx[1] = 0.2f; pc.lpy[1] = 0.6f * up;
            pc.lcAx = 0.0f; pc.lcAy = 0.0f; pc.lcBx = 0.0f; pc.lcBy = 0.0f; pc.rA = 0.01f; pc.rB = 0.01f;
        }
    }
    __syncthreads();
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    int n = w.solver_position_small(is, sh.u.sol.vcs, sh.u.sol.pcs, false, -1, -1, iters);
    if (n < 0) n = w.solver_position_lanes(is, sh.u.sol.vcs, sh.u.sol.pcs, false, -1, -1, iters);
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    __syncthreads();
    if (tid == 0) { out[2 * blockIdx.x] = t1 - t0 + (is.pcx[0] == 12345.0f ? 1ull : 0ull); out[2 * blockIdx.x + 1] = (unsigned long long)n; }
}
}  // namespace
hipError_t mrp::posbench_launch(const EnvTables* all, int nc, int pcount, int iters, int blocks, unsigned long long* d_out) {
    hipError_t e = hipMemcpyToSymbol(HIP_SYMBOL(g_table), all, sizeof(EnvTables));
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(k_posbench, dim3(blocks), dim3(BLOCK), 0, nullptr, nc, pcount, iters, d_out);
    return hipGetLastError();
}
hipError_t mrp::velbench_launch(const EnvTables* all, int nc, int pcount, int iters, int blocks, unsigned long long* d_out) {
    hipError_t e = hipMemcpyToSymbol(HIP_SYMBOL(g_table), all, sizeof(EnvTables));
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(k_velbench, dim3(blocks), dim3(BLOCK), 0, nullptr, nc, pcount, iters, d_out);
    return hipGetLastError();
}
#endif
