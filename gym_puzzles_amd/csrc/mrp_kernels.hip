// mrp_kernels.hip -- gfx950 kernels and the C ABI (include/mrp.h) of libmrp.so.
//
// Execution model: one wavefront (64 threads, one workgroup) owns one world ("lane").  The
// lane's persistent state is contiguous in HBM (lane-major, so the wave moves it with
// coalesced 256-B loads/stores) and lives in LDS for the whole step; order-sensitive Box2D
// work (solver iterations, tree updates, contact-list edits, events) runs on thread 0, while
// the data-parallel phases (SAT narrow phase of every contact, broad-phase pair tests, TOI of
// every candidate contact, state/obs I/O) are spread over the 64 threads.  There is no dense
// contraction in this path, so no MFMA: the work is fp32 VALU with data-dependent control
// flow, plus fp64 for the env-level arithmetic.
#include <hip/hip_runtime.h>

#include <cstddef>
#include <cstdio>
#include <cstring>
#include <new>
#include <string>
#include <vector>

#include "../../include/mrp.h"
#include "mrp_env.h"
#include "mrp_tables.h"

using namespace mrp;

__constant__ EnvTables g_tables[N_ENVS];

#include "mrp_render.h"

namespace {

constexpr int BLOCK = 64;   // one wave per block: lanes of a block never wait on each other

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

// copy this env's hot tables from __constant__ memory into the lane's LDS (before the
// barrier that follows load_state)
template <int ENV>
__device__ __forceinline__ void load_tables(LdsTables<ENV>& L, int tid) {
    using LT = LdsTables<ENV>;
    const EnvTables& T = g_tables[ENV];
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
        Env<ENV> e(sh, g_tables[ENV], P, 0);
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
    const EnvTables& T = g_tables[ENV];
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
    Env<ENV> e(sh, g_tables[ENV], P, tid);
    e.env_reset_coop();
    for (int k = tid; k < D::OBS; k += BLOCK) obs[(size_t)lane * D::OBS + k] = sh.obs[k];
    store_state<ENV>(sh.S, state, lane, tid);
}

template <int ENV>
__global__ __launch_bounds__(BLOCK, 4) void k_step(uint32_t* state, int nl, const float* actions, float* obs, float* reward,
                                                double* reward64, uint8_t* done_out, uint8_t* trunc_out, uint8_t* status_out, float* term_obs,
                                                EnvParams P, uint64_t seed, uint64_t lane_offset, int auto_reset,
                                                int max_steps, const int* __restrict__ order, uint32_t* __restrict__ cost,
                                                const uint32_t* __restrict__ costmax) {
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
    if (tid < 16) sh.trace[tid] = 0;
    long long toi0 = 0, pos0 = 0;
#endif
    load_state<ENV>(sh.S, state, lane, tid);
    load_tables<ENV>(sh.lt, tid);
    __syncthreads();
#ifdef MRP_STAMPS
    toi0 = sh.S.toiEvents; pos0 = sh.S.posIters;
#endif
    MRP_STAMP(0);
    const uint64_t ctr = (uint64_t)sh.S.stepCounter * 64u;
    if (tid < D::ACT)
        sh.act[tid] = actions ? actions[(size_t)lane * D::ACT + tid] : (float)(-1.0 + 2.0 * rng_u01(seed, glane, 3, ctr + tid));
    __syncthreads();
    if (tid == 0) sh.S.stepCounter += 1;
    Env<ENV> e(sh, g_tables[ENV], P, tid);
    if (costmax) {   // priority from the lane's previous-step cost relative to the slowest lane's
        const uint64_t c = cost[lane], m = *costmax;
        e.prio_floor = __builtin_amdgcn_readfirstlane(4 * c > 3 * m ? 3 : (2 * c > m ? 2 : (4 * c > m ? 1 : 0)));
        e.set_prio(e.prio_floor);
    }
    e.env_step_coop();
    if (tid == 0) {
        sh.S.elapsed += 1;
        int d = sh.done, tr = 0;
        if (max_steps > 0 && sh.S.elapsed >= max_steps) { tr = !d; d = 1; }   // gym TimeLimit
        if (reward) reward[lane] = (float)sh.reward;
        if (reward64) reward64[lane] = sh.reward;   // the reference's Python float
        if (done_out) done_out[lane] = (uint8_t)d;
        if (trunc_out) trunc_out[lane] = (uint8_t)tr;
        if (status_out) status_out[lane] = (uint8_t)sh.kind;
        s_fin = d;
    }
    __syncthreads();
    float* orow = obs + (size_t)lane * D::OBS;
    if (term_obs)
        for (int k = tid; k < D::OBS; k += BLOCK) term_obs[(size_t)lane * D::OBS + k] = sh.obs[k];
    MRP_STAMP(8);
    if (s_fin && auto_reset) {   // SB3-style auto-reset with device-RNG spawns
        stage_reset_inputs<ENV>(sh, nullptr, nullptr, lane, tid, seed, glane);
        e.env_reset_coop();
        MRP_STAMP(9);
    }
    for (int k = tid; k < D::OBS; k += BLOCK) orow[k] = sh.obs[k];
    store_state<ENV>(sh.S, state, lane, tid);
    if (cost && tid == 0) cost[lane] = (uint32_t)min(__builtin_amdgcn_s_memtime() - t_start, 0xffffffffull);
    MRP_STAMP(10);
#ifdef MRP_STAMPS
    if (tid == 0) {
        unsigned long long tot = sh.stamp_t - sh.stamp_t0;
        for (int k = 0; k < 11; ++k) { atomicAdd(&g_stamps[k], (unsigned long long)sh.trace[k]); atomicMax(&g_pmax[k], (unsigned long long)sh.trace[k]); }
        atomicAdd(&g_rt[0], tot);
        atomicAdd(&g_rt[1], __builtin_amdgcn_s_memrealtime() - sh.stamp_rt0);
        atomicMax(&g_stepmax[(sh.S.stepCounter - 1u) & 255u], tot);
        sh.trace[11] = (uint32_t)tot;
        sh.trace[13] = (uint32_t)(sh.S.toiEvents - toi0);
        sh.trace[14] = (uint32_t)(sh.S.posIters - pos0);
    }
    __syncthreads();
    if (tid < 16 && lane < 16384) g_trace[lane][tid] = sh.trace[tid];
#endif
}

__global__ __launch_bounds__(256) void k_sincos(const float* x, float* s, float* c, int n) {
    int i = blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    s[i] = g_sinf(x[i]);
    c[i] = g_cosf(x[i]);
}

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

// Dispatch order for the next step: lanes by descending cost of this step (counting sort over 64
// linear buckets of [0, max cost]; order inside a bucket is arbitrary and never affects results).
constexpr int ORDER_NT = 1024, ORDER_NB = 64;
__global__ __launch_bounds__(ORDER_NT) void k_order(const uint32_t* __restrict__ cost, int nl, int* __restrict__ order,
                                                    uint32_t* __restrict__ costmax) {
    __shared__ uint32_t s_max;
    __shared__ int s_cnt[ORDER_NB], s_base[ORDER_NB];
    const int t = threadIdx.x;
    if (t == 0) s_max = 1u;
    if (t < ORDER_NB) s_cnt[t] = 0;
    __syncthreads();
    uint32_t m = 1u;
    for (int l = t; l < nl; l += ORDER_NT) m = max(m, cost[l]);
    atomicMax(&s_max, m);
    __syncthreads();
    const uint64_t mx = s_max;
    if (t == 0 && costmax) *costmax = s_max;
    if (!order) return;
    for (int l = t; l < nl; l += ORDER_NT) {
        const int b = (ORDER_NB - 1) - (int)(((uint64_t)cost[l] * (ORDER_NB - 1)) / mx);   // bucket 0 = costliest
        atomicAdd(&s_cnt[b], 1);
    }
    __syncthreads();
    if (t == 0) {
        int acc = 0;
        for (int b = 0; b < ORDER_NB; ++b) { s_base[b] = acc; acc += s_cnt[b]; }
    }
    __syncthreads();
    for (int l = t; l < nl; l += ORDER_NT) {
        const int b = (ORDER_NB - 1) - (int)(((uint64_t)cost[l] * (ORDER_NB - 1)) / mx);
        order[atomicAdd(&s_base[b], 1)] = l;
    }
}

__global__ __launch_bounds__(256) void k_iota(int* __restrict__ order, int nl) {
    const int l = blockIdx.x * 256 + threadIdx.x;
    if (l < nl) order[l] = l;
}

template <int ENV>
__global__ __launch_bounds__(256) void k_faults(const uint32_t* state, int nl, int32_t* out) {
    const int lane = blockIdx.x * 256 + threadIdx.x;
    if (lane >= nl) return;
    const LaneState<ENV>& S = *reinterpret_cast<const LaneState<ENV>*>(state + (size_t)lane * lane_words<ENV>());
    out[lane] = S.fault;
}

// Diagnostic micro-benchmark of the lane-distributed velocity sweeps (mrp_debug_velbench): a
// synthetic v0 island of nc agent-block contacts with pcount manifold points each, swept `iters`
// times with the early exit off; out[block] = s_memtime cycles of the sweeps.
__global__ __launch_bounds__(BLOCK, 4) void k_velbench(int nc, int pcount, int iters, unsigned long long* out) {
    using W = World<0>;
    __shared__ Shared<0> sh;
    const int tid = threadIdx.x;
    EnvParams P{};
    W w(sh, g_tables[0], P, tid);
    auto& is = sh.isl;
    if (tid == 0) {
        is.nb = nc + 1; is.nc = nc;
        for (int b = 0; b <= nc; ++b) { is.vvx[b] = 0.3f * b - 0.1f; is.vvy[b] = 0.2f - 0.05f * b; is.vw[b] = b == 0 ? 0.01f : 0.0f; }
        for (int i = 0; i < nc; ++i) {
            VC& vc = sh.u.sol.vcs[i];
            const float ang = 0.7f * (float)i + 0.3f;
            vc.nx = __cosf(ang); vc.ny = __sinf(ang);
            vc.iaI = i + 1; vc.ibI = 0; vc.mA = 1.0f; vc.iA = 0.0f; vc.mB = 0.05f; vc.iB = 1.0f / 17.0833f; vc.friction = 0.44f;
            vc.pointCount = pcount;
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

// ------------------------------------------------------------------------------ host side
thread_local std::string g_create_error;

int grid_for(int nl) { return nl; }   // one workgroup (wave) per lane

}  // namespace

struct mrp_ctx {
    int env_id = 0, n_lanes = 0, device = 0;
    uint64_t seed = 0, lane_offset = 0;
    hipStream_t stream = nullptr;
    hipStream_t own_stream = nullptr;
    uint32_t* d_state = nullptr;
    EnvParams params{};
    int auto_reset = 0;
    int schedule = 0;            // dispatch lanes costliest-first (mrp_set_schedule; measured slower, off)
    int* d_order = nullptr;      // [n_lanes] lane stepped by workgroup b
    uint32_t* d_cost = nullptr;  // [n_lanes] last step's cycles per lane
    uint32_t* d_costmax = nullptr;   // max of d_cost (priority mode)
    int have_reset = 0;
    int time_limit = 0;
    double base_puzzle = 10000.0, base_bounds = 1000.0, base_blk_bounds = 100.0;   // set_reward_params
    int shaped_set = 0;                                                             // update_params() called
    int obs_dim = 0, act_dim = 0, n_draws = 0, n_agents = 0, n_blocks = 0, max_steps = 0, words = 0;
    // staging buffers for the host-pointer API
    double* d_draws = nullptr;
    float* d_actions = nullptr;
    uint8_t* d_mask = nullptr;
    float* d_obs = nullptr;
    float* d_reward = nullptr;
    double* d_reward64 = nullptr;
    uint8_t* d_done = nullptr;
    uint8_t* d_trunc = nullptr;
    uint8_t* d_status = nullptr;
    float* d_term = nullptr;
    float* d_bodies = nullptr;
    int32_t* d_flags = nullptr;
    std::string err;
};

#define HIPCHK(ctx, expr)                                                   \
    do {                                                                    \
        hipError_t _e = (expr);                                             \
        if (_e != hipSuccess) {                                             \
            (ctx)->err = std::string(#expr) + ": " + hipGetErrorString(_e); \
            return MRP_E_HIP;                                               \
        }                                                                   \
    } while (0)

#define DISPATCH(env, ...)                                \
    switch (env) {                                        \
    case 0: { constexpr int E = 0; __VA_ARGS__; } break; \
    case 1: { constexpr int E = 1; __VA_ARGS__; } break; \
    case 2: { constexpr int E = 2; __VA_ARGS__; } break; \
    case 3: { constexpr int E = 3; __VA_ARGS__; } break; \
    case 4: { constexpr int E = 4; __VA_ARGS__; } break; \
    case 5: { constexpr int E = 5; __VA_ARGS__; } break; \
    case 6: { constexpr int E = 6; __VA_ARGS__; } break; \
    default: break;                                       \
    }

static int words_for(int env_id) {
    int w = -1;
    DISPATCH(env_id, w = lane_words<E>());
    return w;
}

extern "C" {

int mrp_env_dims(int env_id, int* obs_dim, int* act_dim, int* n_draws, int* n_agents, int* n_blocks, int* max_steps) {
    EnvTables t;
    if (!build_tables(env_id, t)) return MRP_E_ARG;
    if (obs_dim) *obs_dim = t.obs_dim;
    if (act_dim) *act_dim = t.act_dim;
    if (n_draws) *n_draws = t.n_draws;
    if (n_agents) *n_agents = t.n_agents;
    if (n_blocks) *n_blocks = t.n_blocks;
    if (max_steps) *max_steps = t.max_steps;
    return MRP_OK;
}

int mrp_state_words(int env_id) { return words_for(env_id); }

const char* mrp_last_error(const mrp_ctx* ctx) { return ctx ? ctx->err.c_str() : g_create_error.c_str(); }
int mrp_n_lanes(const mrp_ctx* ctx) { return ctx ? ctx->n_lanes : MRP_E_ARG; }
int mrp_env_id(const mrp_ctx* ctx) { return ctx ? ctx->env_id : MRP_E_ARG; }

void mrp_destroy(mrp_ctx* ctx) {
    if (!ctx) return;
    (void)hipSetDevice(ctx->device);
    if (ctx->stream) (void)hipStreamSynchronize(ctx->stream);
    void* bufs[] = {ctx->d_state, ctx->d_draws, ctx->d_actions, ctx->d_mask, ctx->d_obs, ctx->d_reward, ctx->d_reward64,
                    ctx->d_done, ctx->d_trunc, ctx->d_status, ctx->d_term, ctx->d_bodies, ctx->d_flags};
    for (void* p : bufs)
        if (p) (void)hipFree(p);
    if (ctx->d_order) (void)hipFree(ctx->d_order);
    if (ctx->d_cost) (void)hipFree(ctx->d_cost);
    if (ctx->d_costmax) (void)hipFree(ctx->d_costmax);
    if (ctx->own_stream) (void)hipStreamDestroy(ctx->own_stream);
    delete ctx;
}

int mrp_create(int env_id, int n_lanes, int device, uint64_t seed, uint64_t lane_offset, mrp_ctx** out) {
    g_create_error.clear();
    if (!out) { g_create_error = "out is NULL"; return MRP_E_ARG; }
    *out = nullptr;
    EnvTables tables;
    if (!build_tables(env_id, tables)) { g_create_error = "bad env_id"; return MRP_E_ARG; }
    if (n_lanes <= 0) { g_create_error = "n_lanes must be > 0"; return MRP_E_ARG; }
    int ndev = 0;
    hipError_t e = hipGetDeviceCount(&ndev);
    if (e != hipSuccess || ndev <= 0) {
        g_create_error = "no HIP device available (libmrp has no CPU fallback)";
        return MRP_E_HIP;
    }
    if (device < 0 || device >= ndev) { g_create_error = "device index out of range"; return MRP_E_ARG; }
    mrp_ctx* ctx = new (std::nothrow) mrp_ctx();
    if (!ctx) { g_create_error = "out of host memory"; return MRP_E_ARG; }
    ctx->env_id = env_id; ctx->n_lanes = n_lanes; ctx->device = device; ctx->seed = seed; ctx->lane_offset = lane_offset;
    ctx->obs_dim = tables.obs_dim; ctx->act_dim = tables.act_dim; ctx->n_draws = tables.n_draws;
    ctx->n_agents = tables.n_agents; ctx->n_blocks = tables.n_blocks; ctx->max_steps = tables.max_steps;
    ctx->words = words_for(env_id);
    ctx->time_limit = tables.max_steps;
    default_params(env_id, ctx->params);
    auto fail = [&](const char* what, hipError_t he) {
        g_create_error = std::string(what) + ": " + hipGetErrorString(he);
        mrp_destroy(ctx);
        return MRP_E_HIP;
    };
    if ((e = hipSetDevice(device)) != hipSuccess) return fail("hipSetDevice", e);
    EnvTables all[N_ENVS];
    for (int i = 0; i < N_ENVS; ++i) build_tables(i, all[i]);
    if ((e = hipMemcpyToSymbol(HIP_SYMBOL(g_tables), all, sizeof(all))) != hipSuccess) return fail("hipMemcpyToSymbol", e);
    if ((e = hipStreamCreateWithFlags(&ctx->own_stream, hipStreamNonBlocking)) != hipSuccess) return fail("hipStreamCreate", e);
    ctx->stream = ctx->own_stream;
    size_t nl = (size_t)n_lanes;
    struct { void** p; size_t bytes; } allocs[] = {
        {(void**)&ctx->d_state, (size_t)ctx->words * nl * 4},
        {(void**)&ctx->d_draws, nl * ctx->n_draws * sizeof(double)},
        {(void**)&ctx->d_actions, nl * ctx->act_dim * sizeof(float)},
        {(void**)&ctx->d_mask, nl},
        {(void**)&ctx->d_obs, nl * ctx->obs_dim * sizeof(float)},
        {(void**)&ctx->d_term, nl * ctx->obs_dim * sizeof(float)},
        {(void**)&ctx->d_reward, nl * sizeof(float)},
        {(void**)&ctx->d_reward64, nl * sizeof(double)},
        {(void**)&ctx->d_done, nl},
        {(void**)&ctx->d_trunc, nl},
        {(void**)&ctx->d_status, nl},
        {(void**)&ctx->d_bodies, nl * 6 * (ctx->n_agents + ctx->n_blocks) * sizeof(float)},
        {(void**)&ctx->d_flags, nl * (ctx->n_agents + 1) * sizeof(int32_t)},
    };
    for (auto& a : allocs)
        if ((e = hipMalloc(a.p, a.bytes)) != hipSuccess) return fail("hipMalloc", e);
    if ((e = hipMalloc((void**)&ctx->d_order, nl * sizeof(int))) != hipSuccess) return fail("hipMalloc", e);
    if ((e = hipMalloc((void**)&ctx->d_cost, nl * sizeof(uint32_t))) != hipSuccess) return fail("hipMalloc", e);
    if ((e = hipMalloc((void**)&ctx->d_costmax, sizeof(uint32_t))) != hipSuccess) return fail("hipMalloc", e);
    if ((e = hipMemset(ctx->d_cost, 0, nl * sizeof(uint32_t))) != hipSuccess) return fail("hipMemset", e);
    if ((e = hipMemset(ctx->d_costmax, 0xff, sizeof(uint32_t))) != hipSuccess) return fail("hipMemset", e);
    hipLaunchKernelGGL(k_iota, dim3((n_lanes + 255) / 256), dim3(256), 0, ctx->stream, ctx->d_order, n_lanes);
    DISPATCH(env_id, hipLaunchKernelGGL(k_init<E>, dim3(grid_for(n_lanes)), dim3(BLOCK), 0, ctx->stream, ctx->d_state, n_lanes));
    if ((e = hipGetLastError()) != hipSuccess) return fail("k_init launch", e);
    if ((e = hipStreamSynchronize(ctx->stream)) != hipSuccess) return fail("k_init", e);
    *out = ctx;
    return MRP_OK;
}

int mrp_set_stream(mrp_ctx* ctx, void* hip_stream) {
    if (!ctx) return MRP_E_ARG;
    ctx->stream = (hipStream_t)hip_stream;   // NULL: the HIP null stream (torch's default stream)
    return MRP_OK;
}

int mrp_synchronize(mrp_ctx* ctx) {
    if (!ctx) return MRP_E_ARG;
    HIPCHK(ctx, hipSetDevice(ctx->device));
    HIPCHK(ctx, hipStreamSynchronize(ctx->stream));
    return MRP_OK;
}

int mrp_set_reward_params(mrp_ctx* ctx, double agent_delta, double agent_distance, double block_delta, double block_distance,
                          double puzzle_comp, double out_of_bounds, double blk_out_of_bounds) {
    if (!ctx) return MRP_E_ARG;
    ctx->params.w_dAgent = agent_delta; ctx->params.w_agentDist = agent_distance;
    ctx->params.w_dBlock = block_delta; ctx->params.w_blkDist = block_distance;
    ctx->params.puzzle_complete = puzzle_comp;   // v3 step() adds puzzle_complete_reward itself (core.py:408-410)
    ctx->base_puzzle = puzzle_comp; ctx->base_bounds = out_of_bounds; ctx->base_blk_bounds = blk_out_of_bounds;
    // shaped_* are derived only by update_params() (the reference leaves them undefined until
    // then); the batched default before that call is decay = 1, timestep = 0
    if (!ctx->shaped_set) {
        ctx->params.shaped_puzzle = puzzle_comp; ctx->params.shaped_bounds = out_of_bounds;
        ctx->params.shaped_blk_bounds = blk_out_of_bounds;
    }
    return MRP_OK;
}

int mrp_update_params(mrp_ctx* ctx, double timestep, double decay) {
    if (!ctx) return MRP_E_ARG;
    double f = pow(decay, -timestep);   // _02.py:227-230: penalty * decay ** (-timestep)
    ctx->params.shaped_bounds = ctx->base_bounds * f;
    ctx->params.shaped_blk_bounds = ctx->base_blk_bounds * f;
    ctx->params.shaped_puzzle = ctx->base_puzzle * f;
    ctx->shaped_set = 1;
    return MRP_OK;
}

int mrp_update_goal(mrp_ctx* ctx, double epoch, double nb_epochs) {
    if (!ctx) return MRP_E_ARG;
    double eps = (ctx->env_id < 2 || ctx->env_id >= 5) ? 25.0 : 0.1;   // v3 stores it too (core.py:161-162), unused
    ctx->params.scaled_epsilon = eps * (2 - epoch / nb_epochs);
    return MRP_OK;
}

int mrp_set_auto_reset(mrp_ctx* ctx, int enabled) {
    if (!ctx) return MRP_E_ARG;
    ctx->auto_reset = enabled ? 1 : 0;
    return MRP_OK;
}

int mrp_set_time_limit(mrp_ctx* ctx, int max_episode_steps) {
    if (!ctx || max_episode_steps < 0) return MRP_E_ARG;
    ctx->time_limit = max_episode_steps;
    return MRP_OK;
}

int mrp_reset_device(mrp_ctx* ctx, const uint8_t* d_mask, const double* d_draws, const float* d_actions, float* d_obs) {
    if (!ctx || !d_obs) return MRP_E_ARG;
    HIPCHK(ctx, hipSetDevice(ctx->device));
    DISPATCH(ctx->env_id, hipLaunchKernelGGL(k_reset<E>, dim3(grid_for(ctx->n_lanes)), dim3(BLOCK), 0, ctx->stream, ctx->d_state,
                                             ctx->n_lanes, d_mask, d_draws, d_actions, d_obs, ctx->params, ctx->seed,
                                             ctx->lane_offset));
    HIPCHK(ctx, hipGetLastError());
    ctx->have_reset = 1;
    return MRP_OK;
}

int mrp_reset(mrp_ctx* ctx, const uint8_t* mask, const double* draws, const float* actions, float* obs) {
    if (!ctx || !obs) return MRP_E_ARG;
    HIPCHK(ctx, hipSetDevice(ctx->device));
    size_t nl = (size_t)ctx->n_lanes;
    if (mask) HIPCHK(ctx, hipMemcpyAsync(ctx->d_mask, mask, nl, hipMemcpyHostToDevice, ctx->stream));
    if (draws)
        HIPCHK(ctx, hipMemcpyAsync(ctx->d_draws, draws, nl * ctx->n_draws * sizeof(double), hipMemcpyHostToDevice, ctx->stream));
    if (actions)
        HIPCHK(ctx, hipMemcpyAsync(ctx->d_actions, actions, nl * ctx->act_dim * sizeof(float), hipMemcpyHostToDevice, ctx->stream));
    // rows of unmasked lanes stay as the caller had them
    HIPCHK(ctx, hipMemcpyAsync(ctx->d_obs, obs, nl * ctx->obs_dim * sizeof(float), hipMemcpyHostToDevice, ctx->stream));
    int rc = mrp_reset_device(ctx, mask ? ctx->d_mask : nullptr, draws ? ctx->d_draws : nullptr,
                              actions ? ctx->d_actions : nullptr, ctx->d_obs);
    if (rc) return rc;
    HIPCHK(ctx, hipMemcpyAsync(obs, ctx->d_obs, nl * ctx->obs_dim * sizeof(float), hipMemcpyDeviceToHost, ctx->stream));
    HIPCHK(ctx, hipStreamSynchronize(ctx->stream));
    return MRP_OK;
}

int mrp_step_device_ex(mrp_ctx* ctx, const float* d_actions, float* d_obs, float* d_reward, double* d_reward64,
                       uint8_t* d_done, uint8_t* d_trunc, uint8_t* d_status, float* d_term) {
    if (!ctx || !d_obs) return MRP_E_ARG;
    if (!ctx->have_reset) { ctx->err = "step() called before reset()"; return MRP_E_STATE; }
    HIPCHK(ctx, hipSetDevice(ctx->device));
    const int sched = ctx->schedule;
    DISPATCH(ctx->env_id, hipLaunchKernelGGL(k_step<E>, dim3(grid_for(ctx->n_lanes)), dim3(BLOCK), 0, ctx->stream, ctx->d_state,
                                             ctx->n_lanes, d_actions, d_obs, d_reward, d_reward64, d_done, d_trunc, d_status,
                                             d_term, ctx->params, ctx->seed, ctx->lane_offset, ctx->auto_reset,
                                             ctx->time_limit, (sched & 1) ? ctx->d_order : nullptr, sched ? ctx->d_cost : nullptr,
                                             (sched & 2) ? ctx->d_costmax : nullptr));
    HIPCHK(ctx, hipGetLastError());
    if (sched) {   // next step's dispatch order / cost scale (stream-ordered behind this step)
        hipLaunchKernelGGL(k_order, dim3(1), dim3(ORDER_NT), 0, ctx->stream, ctx->d_cost, ctx->n_lanes,
                           (sched & 1) ? ctx->d_order : nullptr, ctx->d_costmax);
        HIPCHK(ctx, hipGetLastError());
    }
    return MRP_OK;
}

int mrp_step_device(mrp_ctx* ctx, const float* d_actions, float* d_obs, float* d_reward, uint8_t* d_done, uint8_t* d_trunc,
                    uint8_t* d_status, float* d_term) {
    return mrp_step_device_ex(ctx, d_actions, d_obs, d_reward, nullptr, d_done, d_trunc, d_status, d_term);
}

int mrp_step_ex(mrp_ctx* ctx, const float* actions, float* obs, float* reward, double* reward64, uint8_t* done, uint8_t* trunc,
                uint8_t* status, float* term) {
    if (!ctx || !obs) return MRP_E_ARG;
    HIPCHK(ctx, hipSetDevice(ctx->device));
    size_t nl = (size_t)ctx->n_lanes;
    if (actions)
        HIPCHK(ctx, hipMemcpyAsync(ctx->d_actions, actions, nl * ctx->act_dim * sizeof(float), hipMemcpyHostToDevice, ctx->stream));
    int rc = mrp_step_device_ex(ctx, actions ? ctx->d_actions : nullptr, ctx->d_obs, ctx->d_reward,
                                reward64 ? ctx->d_reward64 : nullptr, ctx->d_done, ctx->d_trunc, ctx->d_status,
                                term ? ctx->d_term : nullptr);
    if (rc) return rc;
    HIPCHK(ctx, hipMemcpyAsync(obs, ctx->d_obs, nl * ctx->obs_dim * sizeof(float), hipMemcpyDeviceToHost, ctx->stream));
    if (reward) HIPCHK(ctx, hipMemcpyAsync(reward, ctx->d_reward, nl * sizeof(float), hipMemcpyDeviceToHost, ctx->stream));
    if (reward64) HIPCHK(ctx, hipMemcpyAsync(reward64, ctx->d_reward64, nl * sizeof(double), hipMemcpyDeviceToHost, ctx->stream));
    if (done) HIPCHK(ctx, hipMemcpyAsync(done, ctx->d_done, nl, hipMemcpyDeviceToHost, ctx->stream));
    if (trunc) HIPCHK(ctx, hipMemcpyAsync(trunc, ctx->d_trunc, nl, hipMemcpyDeviceToHost, ctx->stream));
    if (status) HIPCHK(ctx, hipMemcpyAsync(status, ctx->d_status, nl, hipMemcpyDeviceToHost, ctx->stream));
    if (term)
        HIPCHK(ctx, hipMemcpyAsync(term, ctx->d_term, nl * ctx->obs_dim * sizeof(float), hipMemcpyDeviceToHost, ctx->stream));
    HIPCHK(ctx, hipStreamSynchronize(ctx->stream));
    return MRP_OK;
}

int mrp_step(mrp_ctx* ctx, const float* actions, float* obs, float* reward, uint8_t* done, uint8_t* trunc, uint8_t* status,
             float* term) {
    return mrp_step_ex(ctx, actions, obs, reward, nullptr, done, trunc, status, term);
}

int mrp_set_schedule(mrp_ctx* ctx, int costliest_first) {
    if (!ctx) return MRP_E_ARG;
    if (costliest_first < 0 || costliest_first > 3) return MRP_E_ARG;
    ctx->schedule = costliest_first;
    return MRP_OK;
}

int mrp_set_seed(mrp_ctx* ctx, uint64_t seed) {
    if (!ctx) return MRP_E_ARG;
    ctx->seed = seed;   // keys every later device-RNG draw; lane state, params, stream and time limit are kept
    return MRP_OK;
}

int mrp_get_bodies(mrp_ctx* ctx, float* out) {
    if (!ctx || !out) return MRP_E_ARG;
    HIPCHK(ctx, hipSetDevice(ctx->device));
    DISPATCH(ctx->env_id, hipLaunchKernelGGL(k_bodies<E>, dim3(grid_for(ctx->n_lanes)), dim3(BLOCK), 0, ctx->stream, ctx->d_state,
                                             ctx->n_lanes, ctx->d_bodies, (int32_t*)nullptr));
    HIPCHK(ctx, hipGetLastError());
    HIPCHK(ctx, hipMemcpyAsync(out, ctx->d_bodies, (size_t)ctx->n_lanes * 6 * (ctx->n_agents + ctx->n_blocks) * sizeof(float),
                               hipMemcpyDeviceToHost, ctx->stream));
    HIPCHK(ctx, hipStreamSynchronize(ctx->stream));
    return MRP_OK;
}

int mrp_get_faults(mrp_ctx* ctx, int32_t* out) {
    if (!ctx || !out) return MRP_E_ARG;
    HIPCHK(ctx, hipSetDevice(ctx->device));
    int32_t* d = (int32_t*)ctx->d_flags;   // [n_lanes][n_agents+1] >= n_lanes words
    DISPATCH(ctx->env_id, hipLaunchKernelGGL(k_faults<E>, dim3((ctx->n_lanes + 255) / 256), dim3(256), 0, ctx->stream,
                                             ctx->d_state, ctx->n_lanes, d));
    HIPCHK(ctx, hipGetLastError());
    HIPCHK(ctx, hipMemcpyAsync(out, d, (size_t)ctx->n_lanes * sizeof(int32_t), hipMemcpyDeviceToHost, ctx->stream));
    HIPCHK(ctx, hipStreamSynchronize(ctx->stream));
    return MRP_OK;
}

int mrp_get_flags(mrp_ctx* ctx, int32_t* out) {
    if (!ctx || !out) return MRP_E_ARG;
    HIPCHK(ctx, hipSetDevice(ctx->device));
    DISPATCH(ctx->env_id, hipLaunchKernelGGL(k_bodies<E>, dim3(grid_for(ctx->n_lanes)), dim3(BLOCK), 0, ctx->stream, ctx->d_state,
                                             ctx->n_lanes, (float*)nullptr, ctx->d_flags));
    HIPCHK(ctx, hipGetLastError());
    HIPCHK(ctx, hipMemcpyAsync(out, ctx->d_flags, (size_t)ctx->n_lanes * (ctx->n_agents + 1) * sizeof(int32_t),
                               hipMemcpyDeviceToHost, ctx->stream));
    HIPCHK(ctx, hipStreamSynchronize(ctx->stream));
    return MRP_OK;
}

int mrp_get_state(mrp_ctx* ctx, uint32_t* out) {
    if (!ctx || !out) return MRP_E_ARG;
    HIPCHK(ctx, hipSetDevice(ctx->device));
    size_t nl = (size_t)ctx->n_lanes, nw = (size_t)ctx->words;
    HIPCHK(ctx, hipMemcpyAsync(out, ctx->d_state, nl * nw * 4, hipMemcpyDeviceToHost, ctx->stream));
    HIPCHK(ctx, hipStreamSynchronize(ctx->stream));
    return MRP_OK;
}

int mrp_set_state(mrp_ctx* ctx, const uint32_t* in) {
    if (!ctx || !in) return MRP_E_ARG;
    HIPCHK(ctx, hipSetDevice(ctx->device));
    size_t nl = (size_t)ctx->n_lanes, nw = (size_t)ctx->words;
    HIPCHK(ctx, hipMemcpyAsync(ctx->d_state, in, nl * nw * 4, hipMemcpyHostToDevice, ctx->stream));
    HIPCHK(ctx, hipStreamSynchronize(ctx->stream));
    ctx->have_reset = 1;
    return MRP_OK;
}

int mrp_counters(mrp_ctx* ctx, int64_t* toi_events, int64_t* pos_iters) {
    if (!ctx) return MRP_E_ARG;
    size_t nl = (size_t)ctx->n_lanes, nw = (size_t)ctx->words;
    std::vector<uint32_t> st(nl * nw);
    int rc = mrp_get_state(ctx, st.data());
    if (rc) return rc;
    size_t off = 0;
    DISPATCH(ctx->env_id, off = offsetof(LaneState<E>, toiEvents) / 4);
    int64_t toi = 0, pos = 0;
    for (size_t l = 0; l < nl; ++l) {
        int64_t a, b;
        std::memcpy(&a, &st[l * nw + off], 8);
        std::memcpy(&b, &st[l * nw + off + 2], 8);
        toi += a; pos += b;
    }
    if (toi_events) *toi_events = toi;
    if (pos_iters) *pos_iters = pos;
    return MRP_OK;
}

// Diagnostic builds only (-DMRP_STAMPS): per-phase thread-0 cycle totals since the last call.
int mrp_debug_progress(int device, uint32_t** host_words, int n_lanes) {
#ifdef MRP_PROGRESS
    if (!host_words || n_lanes <= 0 || hipSetDevice(device) != hipSuccess) return MRP_E_HIP;
    uint32_t* h = nullptr;
    if (hipHostMalloc((void**)&h, (size_t)n_lanes * 4, hipHostMallocMapped) != hipSuccess) return MRP_E_HIP;
    for (int i = 0; i < n_lanes; ++i) h[i] = 0u;
    uint32_t* d = nullptr;
    if (hipHostGetDevicePointer((void**)&d, h, 0) != hipSuccess) return MRP_E_HIP;
    if (hipMemcpyToSymbol(HIP_SYMBOL(g_progress), &d, sizeof(d)) != hipSuccess) return MRP_E_HIP;
    *host_words = h;
    return MRP_OK;
#else
    (void)device; (void)host_words; (void)n_lanes;
    return MRP_E_STATE;
#endif
}

int mrp_debug_velbench(int device, int nc, int pcount, int iters, int blocks, uint64_t* cycles) {
    if (nc < 1 || nc > 16 || pcount < 1 || pcount > 2 || blocks < 1 || !cycles || hipSetDevice(device) != hipSuccess) return MRP_E_ARG;
    EnvTables all[N_ENVS];
    for (int i = 0; i < N_ENVS; ++i) build_tables(i, all[i]);
    if (hipMemcpyToSymbol(HIP_SYMBOL(g_tables), all, sizeof(all)) != hipSuccess) return MRP_E_HIP;
    unsigned long long* d = nullptr;
    if (hipMalloc((void**)&d, (size_t)blocks * 8) != hipSuccess) return MRP_E_HIP;
    hipLaunchKernelGGL(k_velbench, dim3(blocks), dim3(BLOCK), 0, nullptr, nc, pcount, iters, d);
    hipError_t e = hipDeviceSynchronize();
    if (e == hipSuccess) e = hipMemcpy(cycles, d, (size_t)blocks * 8, hipMemcpyDeviceToHost);
    (void)hipFree(d);
    return e == hipSuccess ? MRP_OK : MRP_E_HIP;
}

int mrp_debug_stamps(int device, uint64_t* out16) {
#ifdef MRP_STAMPS
    if (!out16 || hipSetDevice(device) != hipSuccess) return MRP_E_HIP;
    if (hipDeviceSynchronize() != hipSuccess) return MRP_E_HIP;
    if (hipMemcpyFromSymbol(out16, HIP_SYMBOL(g_stamps), 16 * sizeof(uint64_t)) != hipSuccess) return MRP_E_HIP;
    uint64_t z[256] = {0};
    if (hipMemcpyToSymbol(HIP_SYMBOL(g_stamps), z, 16 * sizeof(uint64_t)) != hipSuccess) return MRP_E_HIP;
    return MRP_OK;
#else
    (void)device; (void)out16;
    return MRP_E_STATE;
#endif
}

// Diagnostic builds only: per-phase maxima, per-step slowest-lane totals (256 slots) and the
// (s_memtime, s_memrealtime) sums of lane totals since the last call; all reset afterwards.
int mrp_debug_stamps_ext(int device, uint64_t* pmax16, uint64_t* stepmax256, uint64_t* rt2) {
#ifdef MRP_STAMPS
    if (!pmax16 || !stepmax256 || !rt2 || hipSetDevice(device) != hipSuccess) return MRP_E_HIP;
    if (hipDeviceSynchronize() != hipSuccess) return MRP_E_HIP;
    if (hipMemcpyFromSymbol(pmax16, HIP_SYMBOL(g_pmax), 16 * sizeof(uint64_t)) != hipSuccess) return MRP_E_HIP;
    if (hipMemcpyFromSymbol(stepmax256, HIP_SYMBOL(g_stepmax), 256 * sizeof(uint64_t)) != hipSuccess) return MRP_E_HIP;
    if (hipMemcpyFromSymbol(rt2, HIP_SYMBOL(g_rt), 2 * sizeof(uint64_t)) != hipSuccess) return MRP_E_HIP;
    uint64_t z[256] = {0};
    if (hipMemcpyToSymbol(HIP_SYMBOL(g_pmax), z, 16 * sizeof(uint64_t)) != hipSuccess) return MRP_E_HIP;
    if (hipMemcpyToSymbol(HIP_SYMBOL(g_stepmax), z, 256 * sizeof(uint64_t)) != hipSuccess) return MRP_E_HIP;
    if (hipMemcpyToSymbol(HIP_SYMBOL(g_rt), z, 2 * sizeof(uint64_t)) != hipSuccess) return MRP_E_HIP;
    return MRP_OK;
#else
    (void)device; (void)pmax16; (void)stepmax256; (void)rt2;
    return MRP_E_STATE;
#endif
}

// Diagnostic builds only: the last step's per-lane trace (n_lanes x 16 words, n_lanes <= 16384).
int mrp_debug_trace(int device, uint32_t* out, int n_lanes) {
#ifdef MRP_STAMPS
    if (!out || n_lanes <= 0 || n_lanes > 16384 || hipSetDevice(device) != hipSuccess) return MRP_E_ARG;
    if (hipDeviceSynchronize() != hipSuccess) return MRP_E_HIP;
    if (hipMemcpyFromSymbol(out, HIP_SYMBOL(g_trace), (size_t)n_lanes * 16 * sizeof(uint32_t)) != hipSuccess) return MRP_E_HIP;
    return MRP_OK;
#else
    (void)device; (void)out; (void)n_lanes;
    return MRP_E_STATE;
#endif
}


// ------------------------------------------------------------------------------ rendering
static int render_args(mrp_ctx* ctx, int W, int H, mrpr::RenderArgs& A) {
    if (W <= 0 || H <= 0 || (int64_t)W * H > (1 << 24)) return MRP_E_ARG;
    const bool v0 = ctx->env_id <= 1 || ctx->env_id >= 5;   // v0 and v3 share the 640x480 px / SCALE 30 viewport
    const double ww = v0 ? 640.0 / 30.0 : 1440.0 / 560.0, wh = v0 ? 480.0 / 30.0 : 810.0 / 560.0;
    A.sx = (float)(ww / W); A.sy = (float)(wh / H);
    A.lw_unit = v0 ? (float)(1.0 / 30.0) : (float)(1.0 / 560.0);
    A.ring_r = (float)(ctx->params.scaled_epsilon / (560.0 / 1440.0));
    A.goal_scale = v0 ? 1.0 / 30.0 : 1440.0 / 560.0;
    return MRP_OK;
}

int mrp_render_device(mrp_ctx* ctx, const int32_t* d_lanes, int n, int width, int height, uint8_t* d_rgb) {
    if (!ctx || !d_lanes || !d_rgb || n <= 0 || n > 65535) return MRP_E_ARG;   // n is gridDim.y
    if (!ctx->have_reset) { ctx->err = "mrp_render: call mrp_reset first"; return MRP_E_STATE; }
    mrpr::RenderArgs A;
    if (render_args(ctx, width, height, A) != MRP_OK) { ctx->err = "mrp_render: bad image size"; return MRP_E_ARG; }
    HIPCHK(ctx, hipSetDevice(ctx->device));
    const int per_block = mrpr::RBLOCK * mrpr::RPPT;
    dim3 grid((unsigned)((width * height + per_block - 1) / per_block), (unsigned)n);
    DISPATCH(ctx->env_id, hipLaunchKernelGGL(mrpr::k_render<E>, grid, dim3(mrpr::RBLOCK), 0, ctx->stream, ctx->d_state,
                                             d_lanes, ctx->n_lanes, width, height, A, d_rgb));
    HIPCHK(ctx, hipGetLastError());
    return MRP_OK;
}

int mrp_render(mrp_ctx* ctx, const int32_t* lanes, int n, int width, int height, uint8_t* rgb) {
    if (!ctx || !lanes || !rgb || n <= 0 || width <= 0 || height <= 0) return MRP_E_ARG;
    for (int i = 0; i < n; ++i)
        if (lanes[i] < 0 || lanes[i] >= ctx->n_lanes) { ctx->err = "mrp_render: lane index out of range"; return MRP_E_ARG; }
    HIPCHK(ctx, hipSetDevice(ctx->device));
    int32_t* dl = nullptr; uint8_t* dimg = nullptr;
    const size_t img = (size_t)n * width * height * 3;
    int rc = MRP_E_HIP;
    if (hipMalloc(&dl, n * sizeof(int32_t)) == hipSuccess && hipMalloc(&dimg, img) == hipSuccess &&
        hipMemcpyAsync(dl, lanes, n * sizeof(int32_t), hipMemcpyHostToDevice, ctx->stream) == hipSuccess) {
        rc = mrp_render_device(ctx, dl, n, width, height, dimg);
        if (rc == MRP_OK) {
            rc = MRP_E_HIP;
            if (hipMemcpyAsync(rgb, dimg, img, hipMemcpyDeviceToHost, ctx->stream) == hipSuccess &&
                hipStreamSynchronize(ctx->stream) == hipSuccess)
                rc = MRP_OK;
        }
    }
    if (rc == MRP_E_HIP && ctx->err.empty()) ctx->err = "mrp_render: HIP allocation/copy failed";
    if (dl) (void)hipFree(dl);
    if (dimg) (void)hipFree(dimg);
    return rc;
}

int mrp_get_goals(mrp_ctx* ctx, double* out) {
    if (!ctx || !out) return MRP_E_ARG;
    HIPCHK(ctx, hipSetDevice(ctx->device));
    double* d = nullptr;
    const size_t bytes = (size_t)ctx->n_lanes * ctx->n_blocks * 3 * sizeof(double);
    HIPCHK(ctx, hipMalloc(&d, bytes));
    DISPATCH(ctx->env_id, hipLaunchKernelGGL(mrpr::k_goals<E>, dim3((ctx->n_lanes + 255) / 256), dim3(256), 0, ctx->stream,
                                             ctx->d_state, ctx->n_lanes, d));
    hipError_t e = hipGetLastError();
    if (e == hipSuccess) e = hipMemcpyAsync(out, d, bytes, hipMemcpyDeviceToHost, ctx->stream);
    if (e == hipSuccess) e = hipStreamSynchronize(ctx->stream);
    (void)hipFree(d);
    if (e != hipSuccess) { ctx->err = std::string("mrp_get_goals: ") + hipGetErrorString(e); return MRP_E_HIP; }
    return MRP_OK;
}

int mrp_shapes(int env_id, int32_t* n_fix, int32_t* fix_body, int32_t* counts, float* verts) {
    EnvTables t;
    if (!build_tables(env_id, t) || !n_fix || !fix_body || !counts || !verts) return MRP_E_ARG;
    *n_fix = t.n_fix;
    for (int f = 0; f < MAXF; ++f) {
        fix_body[f] = f < t.n_fix ? t.fix_body[f] : -1;
        counts[f] = f < t.n_fix ? t.shape[f].count : 0;
        for (int i = 0; i < MAX_POLY; ++i) {
            const bool ok = f < t.n_fix && i < t.shape[f].count;
            verts[(f * MAX_POLY + i) * 2] = ok ? t.shape[f].v[i].x : 0.0f;
            verts[(f * MAX_POLY + i) * 2 + 1] = ok ? t.shape[f].v[i].y : 0.0f;
        }
    }
    return MRP_OK;
}

int mrp_selftest_sincos(int device, const float* x, float* sin_out, float* cos_out, int n) {
    if (!x || !sin_out || !cos_out || n <= 0) return MRP_E_ARG;
    if (hipSetDevice(device) != hipSuccess) return MRP_E_HIP;
    float *dx = nullptr, *ds = nullptr, *dc = nullptr;
    size_t bytes = (size_t)n * sizeof(float);
    int rc = MRP_E_HIP;
    if (hipMalloc(&dx, bytes) == hipSuccess && hipMalloc(&ds, bytes) == hipSuccess && hipMalloc(&dc, bytes) == hipSuccess &&
        hipMemcpy(dx, x, bytes, hipMemcpyHostToDevice) == hipSuccess) {
        hipLaunchKernelGGL(k_sincos, dim3((n + 255) / 256), dim3(256), 0, 0, dx, ds, dc, n);
        if (hipGetLastError() == hipSuccess && hipMemcpy(sin_out, ds, bytes, hipMemcpyDeviceToHost) == hipSuccess &&
            hipMemcpy(cos_out, dc, bytes, hipMemcpyDeviceToHost) == hipSuccess)
            rc = MRP_OK;
    }
    if (dx) (void)hipFree(dx);
    if (ds) (void)hipFree(ds);
    if (dc) (void)hipFree(dc);
    return rc;
}

}  // extern "C"
