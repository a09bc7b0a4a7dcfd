// mrp_kernels.hip -- the C ABI (include/mrp.h) of libmrp.so and the env-independent kernels.
//
// The lane kernels of each env id live in their own translation unit (mrp_env<E>.hip, built
// from mrp_lane.h) and are reached through the EnvOps launch table of mrp_ops.h.
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstddef>
#include <cstdio>
#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <new>
#include <string>
#include <vector>

#include "../../include/mrp.h"
#include "mrp_math.h"
#include "mrp_ops.h"
#include "mrp_tables.h"

using namespace mrp;

namespace {
__global__ __launch_bounds__(256) void k_sincos(const float* x, float* s, float* c, int n) {
    int i = blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    const Rot q = rot(x[i]);   // b2Rot::Set as the step evaluates it
    s[i] = q.s;
    c[i] = q.c;
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

// ------------------------------------------------------------------------------ host side
thread_local std::string g_create_error;


}  // namespace

struct mrp_ctx {
    int env_id = 0, n_lanes = 0, device = 0;
    uint64_t seed = 0, lane_offset = 0;
    hipStream_t stream = nullptr;
    hipStream_t own_stream = nullptr;
    uint32_t* d_state = nullptr;
    EnvParams params{};
    int auto_reset = 0;
    int schedule = 0;            // 1: dispatch lanes costliest-first (mrp_set_schedule; default set at mrp_create)
    int* d_order = nullptr;      // [n_lanes] lane stepped by workgroup b
    uint32_t* d_cost = nullptr;  // [n_lanes] last step's cycles per lane
    uint32_t* d_costmax = nullptr;   // max of d_cost (priority mode)
    int have_reset = 0;
    int time_limit = 0;
    double base_puzzle = 10000.0, base_bounds = 1000.0, base_blk_bounds = 100.0;   // set_reward_params
    int shaped_set = 0;                                                             // update_params() called
    int obs_dim = 0, act_dim = 0, n_draws = 0, n_agents = 0, n_blocks = 0, max_steps = 0, words = 0;
    // The host-pointer API's I/O: one pinned, device-mapped host buffer (hipHostMalloc) that the
    // kernels read their inputs from and write their outputs to directly over PCIe, so a host step is
    // one launch and one synchronisation -- no staging copies (the gym-style single env path,
    // train.py:63-80's DummyVecEnv, steps one lane per call).  h_* are host addresses, dev() maps
    // them to the device address of the same bytes.
    uint8_t* h_io = nullptr;
    uint8_t* d_io = nullptr;
    double* h_draws = nullptr;
    float* h_actions = nullptr;
    uint8_t* h_mask = nullptr;
    float* h_obs = nullptr;
    float* h_term = nullptr;
    float* h_reward = nullptr;
    double* h_reward64 = nullptr;
    uint8_t* h_done = nullptr;
    uint8_t* h_trunc = nullptr;
    uint8_t* h_status = nullptr;
    template <class T> T* dev(T* h) const { return h ? reinterpret_cast<T*>(d_io + (reinterpret_cast<uint8_t*>(h) - h_io)) : nullptr; }
    float* d_bodies = nullptr;
    int32_t* d_flags = nullptr;
    int64_t* d_ctr = nullptr;    // [CTR_N] mrp_counters_ex
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

static int words_for(int env_id) {
    const EnvOps* o = env_ops(env_id);
    return o ? o->words : -1;
}

// the host tables and the env's compile-time layout (Dims<ENV> of its unit) describe the same world
static bool layout_matches(int env_id, const EnvTables& t) {
    const EnvOps* o = env_ops(env_id);
    return o && o->dims[0] == t.obs_dim && o->dims[1] == t.act_dim && o->dims[2] == t.n_draws && o->dims[3] == t.n_agents &&
           o->dims[4] == t.n_blocks && o->dims[5] == t.n_fix;
}

extern "C" {

int mrp_env_dims(int env_id, int* obs_dim, int* act_dim, int* n_draws, int* n_agents, int* n_blocks, int* max_steps) {
    EnvTables t;
    if (!build_tables(env_id, t)) return MRP_E_ARG;
    if (!layout_matches(env_id, t)) return MRP_E_STATE;
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
    void* bufs[] = {ctx->d_state, ctx->d_bodies, ctx->d_flags, ctx->d_ctr};
    for (void* p : bufs)
        if (p) (void)hipFree(p);
    if (ctx->h_io) (void)hipHostFree(ctx->h_io);
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
    if (!layout_matches(env_id, tables)) {
        g_create_error = "env tables disagree with the compiled layout of env_id " + std::to_string(env_id);
        return MRP_E_STATE;
    }
    if (n_lanes <= 0) { g_create_error = "n_lanes must be > 0"; return MRP_E_ARG; }
    // the velocity solver drops the (then identically +0) restitution velocity bias (mrp_world.h CC):
    // every fixture of every env has the default restitution 0 (no reference fixtureDef sets one)
    for (int f = 0; f < tables.n_fix; ++f)
        if (tables.fix_restitution[f] != 0.0f) { g_create_error = "fixture restitution != 0 is not supported"; return MRP_E_ARG; }
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
    {   // lanes beyond the first resident set of k_step waves start as earlier ones finish; where
        // there are such lanes, Heavy-v0 and v3 dispatch the previous step's costliest lanes first
        // (round 4 A/B, profiles/r4_ab_paired_sweeps_schedule.txt: Heavy-v0 +4 % in the driver
        // window and +10 % at steps 21-220, v3 +1-2 %; v0 -0.9 % / +1 %, and -3..-5 % at 1024
        // lanes, where every lane is resident and only the ordering kernel's cost remains)
        int cus = 0;
        if ((e = hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, device)) != hipSuccess)
            return fail("hipDeviceGetAttribute", e);
        const int resident = cus * 4 * env_ops(env_id)->step_waves_per_eu;
        if ((env_id == 1 || env_id == 5) && n_lanes > resident) ctx->schedule = 1;
    }
    EnvTables all[N_ENVS];
    for (int i = 0; i < N_ENVS; ++i) build_tables(i, all[i]);
    for (int i = 0; i < N_ENVS; ++i)   // every unit keeps its own __constant__ copy
        if ((e = env_ops(i)->upload_tables(all)) != hipSuccess) return fail("hipMemcpyToSymbol", e);
    if ((e = hipStreamCreateWithFlags(&ctx->own_stream, hipStreamNonBlocking)) != hipSuccess) return fail("hipStreamCreate", e);
    ctx->stream = ctx->own_stream;
    size_t nl = (size_t)n_lanes;
    struct { void** p; size_t bytes; } allocs[] = {
        {(void**)&ctx->d_state, (size_t)ctx->words * nl * 4},
        {(void**)&ctx->d_bodies, nl * 6 * (ctx->n_agents + ctx->n_blocks) * sizeof(float)},
        {(void**)&ctx->d_flags, nl * (ctx->n_agents + 1) * sizeof(int32_t)},
        {(void**)&ctx->d_ctr, CTR_N * sizeof(int64_t)},
    };
    // MRP_STATE_ALLOC=contiguous (diagnostic A/B): the lane state as one physically contiguous
    // allocation (large page fragments, so the GPU TLB covers it with few entries)
    const char* pol = std::getenv("MRP_STATE_ALLOC");
    const bool contiguous = pol && std::strcmp(pol, "contiguous") == 0;
    for (auto& a : allocs) {
        if (contiguous && a.p == (void**)&ctx->d_state) e = hipExtMallocWithFlags(a.p, a.bytes, hipDeviceMallocContiguous);
        else e = hipMalloc(a.p, a.bytes);
        if (e != hipSuccess) return fail("hipMalloc", e);
    }
    {   // the host API's pinned I/O buffer, carved 16-B aligned: doubles first, then floats, then bytes
        auto up = [](size_t b) { return (b + 15) & ~(size_t)15; };
        const size_t sz_draws = up(nl * ctx->n_draws * sizeof(double)), sz_r64 = up(nl * sizeof(double));
        const size_t sz_act = up(nl * ctx->act_dim * sizeof(float)), sz_obs = up(nl * ctx->obs_dim * sizeof(float));
        const size_t sz_rew = up(nl * sizeof(float)), sz_b = up(nl);
        const size_t bytes = sz_draws + sz_r64 + sz_act + 2 * sz_obs + sz_rew + 4 * sz_b;
        if ((e = hipHostMalloc((void**)&ctx->h_io, bytes, hipHostMallocMapped | hipHostMallocCoherent)) != hipSuccess)
            return fail("hipHostMalloc", e);
        if ((e = hipHostGetDevicePointer((void**)&ctx->d_io, ctx->h_io, 0)) != hipSuccess) return fail("hipHostGetDevicePointer", e);
        std::memset(ctx->h_io, 0, bytes);
        uint8_t* q = ctx->h_io;
        ctx->h_draws = (double*)q; q += sz_draws;
        ctx->h_reward64 = (double*)q; q += sz_r64;
        ctx->h_actions = (float*)q; q += sz_act;
        ctx->h_obs = (float*)q; q += sz_obs;
        ctx->h_term = (float*)q; q += sz_obs;
        ctx->h_reward = (float*)q; q += sz_rew;
        ctx->h_mask = q; q += sz_b;
        ctx->h_done = q; q += sz_b;
        ctx->h_trunc = q; q += sz_b;
        ctx->h_status = q;
    }
    if ((e = hipMalloc((void**)&ctx->d_order, nl * sizeof(int))) != hipSuccess) return fail("hipMalloc", e);
    if ((e = hipMalloc((void**)&ctx->d_cost, nl * sizeof(uint32_t))) != hipSuccess) return fail("hipMalloc", e);
    if ((e = hipMalloc((void**)&ctx->d_costmax, sizeof(uint32_t))) != hipSuccess) return fail("hipMalloc", e);
    if ((e = hipMemset(ctx->d_cost, 0, nl * sizeof(uint32_t))) != hipSuccess) return fail("hipMemset", e);
    if ((e = hipMemset(ctx->d_costmax, 0xff, sizeof(uint32_t))) != hipSuccess) return fail("hipMemset", e);
    hipLaunchKernelGGL(k_iota, dim3((n_lanes + 255) / 256), dim3(256), 0, ctx->stream, ctx->d_order, n_lanes);
    env_ops(env_id)->init(ctx->stream, ctx->d_state, n_lanes);
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
    double eps = ENV_CFG[ctx->env_id].version != 2 ? 25.0 : 0.1;   // v3 stores it too (core.py:161-162), unused
    ctx->params.scaled_epsilon = eps * (2 - epoch / nb_epochs);
    return MRP_OK;
}

int mrp_set_frameskip(mrp_ctx* ctx, int frameskip) {
    if (!ctx || frameskip < 1 || frameskip > 64) return MRP_E_ARG;
    ctx->params.frameskip = frameskip;
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
    env_ops(ctx->env_id)->reset(ctx->stream, ctx->d_state, ctx->n_lanes, d_mask, d_draws, d_actions, d_obs, ctx->params,
                                ctx->seed, ctx->lane_offset);
    HIPCHK(ctx, hipGetLastError());
    ctx->have_reset = 1;
    return MRP_OK;
}

int mrp_reset(mrp_ctx* ctx, const uint8_t* mask, const double* draws, const float* actions, float* obs) {
    if (!ctx || !obs) return MRP_E_ARG;
    HIPCHK(ctx, hipSetDevice(ctx->device));
    size_t nl = (size_t)ctx->n_lanes;
    // inputs into the pinned I/O buffer; the kernel reads them and writes the reset rows there
    if (mask) std::memcpy(ctx->h_mask, mask, nl);
    if (draws) std::memcpy(ctx->h_draws, draws, nl * ctx->n_draws * sizeof(double));
    if (actions) std::memcpy(ctx->h_actions, actions, nl * ctx->act_dim * sizeof(float));
    // rows of unmasked lanes stay as the caller had them
    if (mask) std::memcpy(ctx->h_obs, obs, nl * ctx->obs_dim * sizeof(float));
    int rc = mrp_reset_device(ctx, mask ? ctx->dev(ctx->h_mask) : nullptr, draws ? ctx->dev(ctx->h_draws) : nullptr,
                              actions ? ctx->dev(ctx->h_actions) : nullptr, ctx->dev(ctx->h_obs));
    if (rc) return rc;
    HIPCHK(ctx, hipStreamSynchronize(ctx->stream));
    std::memcpy(obs, ctx->h_obs, nl * ctx->obs_dim * sizeof(float));
    return MRP_OK;
}

static_assert(MRP_STATUS_NONFINITE == MRP_STATUS_NONFINITE_BIT && MRP_STATUS_FAULT == MRP_STATUS_FAULT_BIT,
              "status flag bits of include/mrp.h and the kernels agree");

static int step_launch(mrp_ctx* ctx, int n_steps, const float* d_actions, float* d_obs, float* d_reward, double* d_reward64,
                       uint8_t* d_done, uint8_t* d_trunc, uint8_t* d_status, float* d_term) {
    if (!ctx || !d_obs || n_steps < 1) return MRP_E_ARG;
    if (!ctx->have_reset) { ctx->err = "step() called before reset()"; return MRP_E_STATE; }
    HIPCHK(ctx, hipSetDevice(ctx->device));
    const int sched = ctx->schedule;
    StepArgs a{ctx->d_state, ctx->n_lanes, d_actions, d_obs, d_reward, d_reward64, d_done, d_trunc, d_status, d_term,
               ctx->params, ctx->seed, ctx->lane_offset, ctx->auto_reset, ctx->time_limit,
               (sched & 1) ? ctx->d_order : nullptr, sched ? ctx->d_cost : nullptr, (sched & 2) ? ctx->d_costmax : nullptr,
               n_steps};
    env_ops(ctx->env_id)->step(ctx->stream, a);
    HIPCHK(ctx, hipGetLastError());
    if (sched) {   // next step's dispatch order / cost scale (stream-ordered behind this step)
        hipLaunchKernelGGL(k_order, dim3(1), dim3(ORDER_NT), 0, ctx->stream, ctx->d_cost, ctx->n_lanes,
                           (sched & 1) ? ctx->d_order : nullptr, ctx->d_costmax);
        HIPCHK(ctx, hipGetLastError());
    }
    return MRP_OK;
}

int mrp_step_device_ex(mrp_ctx* ctx, const float* d_actions, float* d_obs, float* d_reward, double* d_reward64,
                       uint8_t* d_done, uint8_t* d_trunc, uint8_t* d_status, float* d_term) {
    return step_launch(ctx, 1, d_actions, d_obs, d_reward, d_reward64, d_done, d_trunc, d_status, d_term);
}

int mrp_step_n_device(mrp_ctx* ctx, int n_steps, const float* d_actions, float* d_obs, float* d_reward, double* d_reward64,
                      uint8_t* d_done, uint8_t* d_trunc, uint8_t* d_status, float* d_term) {
    if (ctx && n_steps < 1) { ctx->err = "mrp_step_n_device: n_steps must be >= 1"; return MRP_E_ARG; }
    return step_launch(ctx, n_steps, d_actions, d_obs, d_reward, d_reward64, d_done, d_trunc, d_status, d_term);
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
    // one launch that reads the actions from and writes every output into the pinned I/O buffer,
    // one synchronisation, then host copies out of it
    if (actions) std::memcpy(ctx->h_actions, actions, nl * ctx->act_dim * sizeof(float));
    int rc = mrp_step_device_ex(ctx, actions ? ctx->dev(ctx->h_actions) : nullptr, ctx->dev(ctx->h_obs),
                                reward ? ctx->dev(ctx->h_reward) : nullptr, reward64 ? ctx->dev(ctx->h_reward64) : nullptr,
                                done ? ctx->dev(ctx->h_done) : nullptr, trunc ? ctx->dev(ctx->h_trunc) : nullptr,
                                status ? ctx->dev(ctx->h_status) : nullptr, term ? ctx->dev(ctx->h_term) : nullptr);
    if (rc) return rc;
    HIPCHK(ctx, hipStreamSynchronize(ctx->stream));
    std::memcpy(obs, ctx->h_obs, nl * ctx->obs_dim * sizeof(float));
    if (reward) std::memcpy(reward, ctx->h_reward, nl * sizeof(float));
    if (reward64) std::memcpy(reward64, ctx->h_reward64, nl * sizeof(double));
    if (done) std::memcpy(done, ctx->h_done, nl);
    if (trunc) std::memcpy(trunc, ctx->h_trunc, nl);
    if (status) std::memcpy(status, ctx->h_status, nl);
    if (term) std::memcpy(term, ctx->h_term, nl * ctx->obs_dim * sizeof(float));
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
int mrp_get_schedule(const mrp_ctx* ctx) { return ctx ? ctx->schedule : MRP_E_ARG; }

int mrp_set_seed(mrp_ctx* ctx, uint64_t seed) {
    if (!ctx) return MRP_E_ARG;
    ctx->seed = seed;   // keys every later device-RNG draw; lane state, params, stream and time limit are kept
    return MRP_OK;
}

int mrp_get_bodies(mrp_ctx* ctx, float* out) {
    if (!ctx || !out) return MRP_E_ARG;
    HIPCHK(ctx, hipSetDevice(ctx->device));
    env_ops(ctx->env_id)->bodies(ctx->stream, ctx->d_state, ctx->n_lanes, ctx->d_bodies, nullptr);
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
    env_ops(ctx->env_id)->faults(ctx->stream, ctx->d_state, ctx->n_lanes, d);
    HIPCHK(ctx, hipGetLastError());
    HIPCHK(ctx, hipMemcpyAsync(out, d, (size_t)ctx->n_lanes * sizeof(int32_t), hipMemcpyDeviceToHost, ctx->stream));
    HIPCHK(ctx, hipStreamSynchronize(ctx->stream));
    return MRP_OK;
}

int mrp_get_flags(mrp_ctx* ctx, int32_t* out) {
    if (!ctx || !out) return MRP_E_ARG;
    HIPCHK(ctx, hipSetDevice(ctx->device));
    env_ops(ctx->env_id)->bodies(ctx->stream, ctx->d_state, ctx->n_lanes, nullptr, ctx->d_flags);
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
    // k_step moves only the contact slots below a lane's high-water mark cHW and rebuilds the rest
    // in LDS with their initial contents (mrp_lane.h StateIO), so a state whose cHW understates its
    // highest non-initial slot would lose contacts silently.  Recompute the mark from the slots:
    // 1 + the highest slot whose words differ from the initial ones (cnext[c] = c + 1 or NULL, every
    // other array 0), never lower than the stored value (a higher mark only moves more words).
    const EnvOps* o = env_ops(ctx->env_id);
    std::vector<uint32_t> st(in, in + nl * nw);
    const size_t C = (size_t)o->cslot_n;
    for (size_t l = 0; l < nl; ++l) {
        uint32_t* w = st.data() + l * nw;
        int hw = 0;
        for (size_t a = 0; a < (size_t)o->cslot_arrays; ++a)
            for (size_t c = (size_t)hw; c < C; ++c) {
                const uint32_t init = a == 0 ? (c + 1 < C ? (uint32_t)(c + 1) : 0xffffffffu) : 0u;
                if (w[o->cslot_word + a * C + c] != init) hw = (int)c + 1;
            }
        int32_t mark;
        std::memcpy(&mark, &w[o->chw_word], 4);
        mark = std::max(std::min(mark, (int32_t)C), (int32_t)hw);
        std::memcpy(&w[o->chw_word], &mark, 4);
    }
    HIPCHK(ctx, hipMemcpyAsync(ctx->d_state, st.data(), nl * nw * 4, hipMemcpyHostToDevice, ctx->stream));
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
    off = (size_t)env_ops(ctx->env_id)->counters_word;
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

int mrp_counters_ex(mrp_ctx* ctx, int64_t* out8) {
    if (!ctx || !out8) return MRP_E_ARG;
    HIPCHK(ctx, hipSetDevice(ctx->device));
    env_ops(ctx->env_id)->counters(ctx->stream, ctx->d_state, ctx->n_lanes, ctx->d_ctr);
    HIPCHK(ctx, hipGetLastError());
    HIPCHK(ctx, hipMemcpyAsync(out8, ctx->d_ctr, CTR_N * sizeof(int64_t), hipMemcpyDeviceToHost, ctx->stream));
    HIPCHK(ctx, hipStreamSynchronize(ctx->stream));
    return MRP_OK;
}

// Diagnostic builds only (-DMRP_STAMPS): per-phase thread-0 cycle totals since the last call.
int mrp_debug_progress(int device, uint32_t** host_words, int n_lanes) {
    if (!host_words || n_lanes <= 0 || hipSetDevice(device) != hipSuccess) return MRP_E_HIP;
    if (env_ops(0)->debug_progress(nullptr) == hipErrorNotSupported) return MRP_E_STATE;   // not a -DMRP_PROGRESS build
    uint32_t* h = nullptr;
    if (hipHostMalloc((void**)&h, (size_t)n_lanes * 4, hipHostMallocMapped) != hipSuccess) return MRP_E_HIP;
    for (int i = 0; i < n_lanes; ++i) h[i] = 0u;
    uint32_t* d = nullptr;
    if (hipHostGetDevicePointer((void**)&d, h, 0) != hipSuccess) return MRP_E_HIP;
    for (int i = 0; i < N_ENVS; ++i)
        if (env_ops(i)->debug_progress(d) != hipSuccess) return MRP_E_HIP;
    *host_words = h;
    return MRP_OK;
}

int mrp_debug_velbench(int device, int nc, int pcount, int iters, int blocks, uint64_t* cycles) {
    const int ncc = nc >= 100 ? nc - 100 : nc;   // nc >= 100: a chain of nc - 100 contacts (k_velbench); ncc + 1 bodies <= v0's 7
    if (ncc < 1 || ncc > 6 || pcount < 1 || pcount > 2 || blocks < 1 || !cycles || hipSetDevice(device) != hipSuccess) return MRP_E_ARG;
    EnvTables all[N_ENVS];
    for (int i = 0; i < N_ENVS; ++i) build_tables(i, all[i]);
    unsigned long long* d = nullptr;
    if (hipMalloc((void**)&d, (size_t)blocks * 8) != hipSuccess) return MRP_E_HIP;
    hipError_t e = velbench_launch(all, nc, pcount, iters, blocks, d);
    if (e == hipSuccess) e = hipDeviceSynchronize();
    if (e == hipSuccess) e = hipMemcpy(cycles, d, (size_t)blocks * 8, hipMemcpyDeviceToHost);
    (void)hipFree(d);
    return e == hipSuccess ? MRP_OK : MRP_E_HIP;
}

int mrp_debug_posbench(int device, int nc, int pcount, int iters, int blocks, uint64_t* out) {
    if (nc < 1 || nc > 6 || pcount < 1 || pcount > 2 || iters < 1 || blocks < 1 || !out || hipSetDevice(device) != hipSuccess)
        return MRP_E_ARG;
    EnvTables all[N_ENVS];
    for (int i = 0; i < N_ENVS; ++i) build_tables(i, all[i]);
    unsigned long long* d = nullptr;
    if (hipMalloc((void**)&d, (size_t)blocks * 16) != hipSuccess) return MRP_E_HIP;
    hipError_t e = posbench_launch(all, nc, pcount, iters, blocks, d);
    if (e == hipSuccess) e = hipDeviceSynchronize();
    if (e == hipSuccess) e = hipMemcpy(out, d, (size_t)blocks * 16, hipMemcpyDeviceToHost);
    (void)hipFree(d);
    return e == hipSuccess ? MRP_OK : MRP_E_HIP;
}

// Diagnostic builds only: read-and-clear one stamp symbol of every env unit, combined by sum
// (or max); only the units whose kernels ran hold non-zero values.
// A variant library (build.py --variant ... -DMRP_STAMPS) instruments only the env units it lists;
// units without the stamps are skipped, and a library with none answers MRP_E_STATE.
static int debug_combine(int what, uint64_t* out, size_t n, bool take_max) {
    std::vector<uint64_t> tmp(n);
    for (size_t k = 0; k < n; ++k) out[k] = 0;
    int have = 0;
    for (int i = 0; i < N_ENVS; ++i) {
        hipError_t e = env_ops(i)->debug_read(what, tmp.data(), n * sizeof(uint64_t));
        if (e == hipErrorNotSupported) continue;
        if (e != hipSuccess) return MRP_E_HIP;
        ++have;
        for (size_t k = 0; k < n; ++k) out[k] = take_max ? std::max(out[k], tmp[k]) : out[k] + tmp[k];
    }
    return have ? MRP_OK : MRP_E_STATE;
}

int mrp_debug_stamps(int device, uint64_t* out16) {
    if (!out16 || hipSetDevice(device) != hipSuccess) return MRP_E_HIP;
    return debug_combine(DBG_STAMPS, out16, 16, false);
}

// Diagnostic builds only: per-phase maxima, per-step slowest-lane totals (256 slots) and the
// (s_memtime, s_memrealtime) sums of lane totals since the last call; all reset afterwards.
int mrp_debug_stamps_ext(int device, uint64_t* pmax16, uint64_t* stepmax256, uint64_t* rt2) {
    if (!pmax16 || !stepmax256 || !rt2 || hipSetDevice(device) != hipSuccess) return MRP_E_HIP;
    int rc = debug_combine(DBG_PMAX, pmax16, 16, true);
    if (rc == MRP_OK) rc = debug_combine(DBG_STEPMAX, stepmax256, 256, true);
    if (rc == MRP_OK) rc = debug_combine(DBG_RT, rt2, 2, false);
    return rc;
}

// Diagnostic builds only: the last step's per-lane trace (n_lanes x MRP_TRACE_WORDS words,
// n_lanes <= 16384).  The width is the stamps build's trace row (mrp_lane.h g_trace); callers size
// their buffer from mrp_debug_trace_words() so the two cannot drift apart.
int mrp_debug_trace_words(void) { return MRP_TRACE_WORDS; }
int mrp_debug_trace(int device, uint32_t* out, int n_lanes) {
    if (!out || n_lanes <= 0 || n_lanes > 16384 || hipSetDevice(device) != hipSuccess) return MRP_E_ARG;
    std::vector<uint32_t> tmp((size_t)n_lanes * MRP_TRACE_WORDS);
    int have = 0;
    for (int i = 0; i < N_ENVS; ++i) {   // only the unit that stepped has a non-zero trace
        hipError_t e = env_ops(i)->debug_read(DBG_TRACE, tmp.data(), tmp.size() * 4);
        if (e == hipErrorNotSupported) continue;
        if (e != hipSuccess) return MRP_E_HIP;
        if (!have) std::memset(out, 0, tmp.size() * 4);   // the caller's buffer is written only by a stamps build
        ++have;
        for (size_t k = 0; k < tmp.size(); ++k) out[k] |= tmp[k];
    }
    return have ? MRP_OK : MRP_E_STATE;
}


// ------------------------------------------------------------------------------ rendering
static int render_args(mrp_ctx* ctx, int W, int H, mrpr::RenderArgs& A) {
    if (W <= 0 || H <= 0 || (int64_t)W * H > (1 << 24)) return MRP_E_ARG;
    const bool v0 = ENV_CFG[ctx->env_id].version != 2;   // v0 and v3 share the 640x480 px / SCALE 30 viewport
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
    env_ops(ctx->env_id)->render(ctx->stream, grid, ctx->d_state, d_lanes, ctx->n_lanes, width, height, A, d_rgb);
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
    env_ops(ctx->env_id)->goals(ctx->stream, ctx->d_state, ctx->n_lanes, d);
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
