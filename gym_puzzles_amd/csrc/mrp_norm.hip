// mrp_norm.hip -- on-device VecNormalize + Monitor statistics for a batch of lanes (SURVEY.md
// 8f-2).  The reference trains with stable-baselines3's Monitor(env) per env and
// VecNormalize(DummyVecEnv(...)) with default arguments (train/train.py:68,80-82; reloaded by
// train/test.py:66); this is the same arithmetic on the step outputs while they are still in
// HBM, so a policy on the GPU never sees host copies.
//
// Semantics (stable-baselines3 1.x VecNormalize / RunningMeanStd / Monitor, restated):
//   reset : obs_rms.update(obs) (training), obs' = clip((obs - mean) / sqrt(var + eps), +-clip_obs)
//   step  : obs_rms.update(obs); obs' as above; returns = returns * gamma + reward;
//           ret_rms.update(returns); reward' = clip(reward / sqrt(ret_var + eps), +-clip_reward);
//           terminal_obs' normalised with the updated obs_rms; returns[done] = 0.
//   RunningMeanStd.update(x[L][D]) (Chan et al. parallel moments): batch mean/var over the L
//   lanes, delta = bm - mean, tot = count + L, mean += delta * L / tot,
//   var = (var * count + bv * L + delta^2 * count * L / tot) / tot, count = tot.
//   Monitor: per lane ep_return += reward (float64, in step order), ep_len += 1; on done both
//   are reported and restarted.
// The batch moments are float64 (two passes over the lanes); numpy's float32 np.mean/np.var
// of a float32 batch round differently, so parity with the restatement is to a stated
// tolerance (tests/test_norm.py), not bitwise.  Monitor sums are bit-exact.
//
// Kernels: k_moments (one block per statistic column: the D obs columns, plus one block that
// advances the per-lane discounted returns and takes their moments) and k_apply (one thread per
// obs element for the normalised obs / terminal obs; per lane: reward, returns reset, Monitor).
// Both are tiny next to k_step; the statistics stay on the device between steps.
#include <hip/hip_runtime.h>

#include <cmath>
#include <new>
#include <string>

#include "../../include/mrp.h"

namespace {

constexpr int NT = 256;

__device__ __forceinline__ double block_sum(double v, double* red) {
    const int t = threadIdx.x;
    red[t] = v;
    __syncthreads();
    for (int s = NT / 2; s > 0; s >>= 1) {
        if (t < s) red[t] += red[t + s];
        __syncthreads();
    }
    double r = red[0];
    __syncthreads();
    return r;
}

// Chan et al. merge of the batch moments (mean, var over n) into the running (mean, var, count)
__device__ __forceinline__ void rms_merge(double* mean, double* var, double* count, double bm, double bv, double n) {
    double delta = bm - *mean;
    double tot = *count + n;
    double new_mean = *mean + delta * n / tot;
    double m_a = *var * *count;
    double m_b = bv * n;
    double m2 = m_a + m_b + delta * delta * *count * n / tot;
    *mean = new_mean;
    *var = m2 / tot;
    *count = tot;
}

// blocks 0..D-1: obs column moments (if update_obs); block D: returns update + moments (if step)
__global__ __launch_bounds__(NT) void k_moments(const float* __restrict__ obs, int L, int D, const float* __restrict__ reward,
                                                double* __restrict__ returns, double gamma, double* obs_mean, double* obs_var,
                                                double* obs_count, double* ret_stats, int update_obs, int step) {
    __shared__ double red[NT];
    const int col = blockIdx.x, t = threadIdx.x;
    const double n = (double)L;
    if (col < D) {
        if (!update_obs) return;
        double s = 0.0;
        for (int l = t; l < L; l += NT) s += (double)obs[(size_t)l * D + col];
        const double bm = block_sum(s, red) / n;
        double q = 0.0;
        for (int l = t; l < L; l += NT) { double d = (double)obs[(size_t)l * D + col] - bm; q += d * d; }
        const double bv = block_sum(q, red) / n;
        if (t == 0) {
            double c = *obs_count;   // every column block reads the pre-update count
            double m = obs_mean[col], v = obs_var[col];
            rms_merge(&m, &v, &c, bm, bv, n);
            obs_mean[col] = m; obs_var[col] = v;
        }
    } else {
        if (!step) return;
        double s = 0.0;
        for (int l = t; l < L; l += NT) {
            double r = returns[l] * gamma + (double)reward[l];
            returns[l] = r;
            s += r;
        }
        const double bm = block_sum(s, red) / n;
        double q = 0.0;
        for (int l = t; l < L; l += NT) { double d = returns[l] - bm; q += d * d; }
        const double bv = block_sum(q, red) / n;
        if (t == 0) rms_merge(&ret_stats[0], &ret_stats[1], &ret_stats[2], bm, bv, n);
    }
}

// one thread per obs element (coalesced rows) for obs / terminal obs; threads e < L also do lane
// e's reward, discounted-return reset and Monitor accumulators; thread 0 advances the obs count
// (k_moments read the pre-update count)
__global__ __launch_bounds__(NT) void k_apply(const float* __restrict__ obs, const float* __restrict__ term, int L, int D,
                                              const double* __restrict__ obs_mean, const double* __restrict__ obs_var,
                                              double* __restrict__ obs_count, int count_obs,
                                              const double* __restrict__ ret_stats, double clip_obs, double clip_rew, double eps,
                                              const float* __restrict__ reward, const double* __restrict__ reward64,
                                              const uint8_t* __restrict__ done, double* __restrict__ returns, float* __restrict__ obs_out, float* __restrict__ term_out,
                                              float* __restrict__ reward_out, double* __restrict__ ep_ret, int* __restrict__ ep_len,
                                              double* __restrict__ ep_ret_out, int* __restrict__ ep_len_out, int step) {
    const int e = blockIdx.x * NT + threadIdx.x;
    if (e == 0 && count_obs) *obs_count += (double)L;
    if (e < L * D) {
        const int l = e / D, j = e - l * D;
        const double sd = sqrt(obs_var[j] + eps);
        double x = ((double)obs[e] - obs_mean[j]) / sd;
        obs_out[e] = (float)fmin(fmax(x, -clip_obs), clip_obs);
        if (step && done && done[l] && term && term_out) {
            double y = ((double)term[e] - obs_mean[j]) / sd;
            term_out[e] = (float)fmin(fmax(y, -clip_obs), clip_obs);
        }
    }
    if (e >= L) return;
    const int l = e;
    if (!step) { returns[l] = 0.0; ep_ret[l] = 0.0; ep_len[l] = 0; return; }
    const bool fin = done && done[l];
    const double r = (double)reward[l];
    if (reward_out) {
        double x = r / sqrt(ret_stats[1] + eps);
        reward_out[l] = (float)fmin(fmax(x, -clip_rew), clip_rew);
    }
    // Monitor sums the env's own (float64) rewards when the step exported them
    double er = ep_ret[l] + (reward64 ? reward64[l] : r);
    int el = ep_len[l] + 1;
    if (fin) {
        returns[l] = 0.0;
        if (ep_ret_out) ep_ret_out[l] = er;
        if (ep_len_out) ep_len_out[l] = el;
        er = 0.0; el = 0;
    }
    ep_ret[l] = er; ep_len[l] = el;
}

thread_local std::string g_norm_create_error;

}  // namespace

struct mrp_norm {
    int n_lanes = 0, obs_dim = 0, device = 0, training = 1, norm_obs = 1;
    double clip_obs = 10.0, clip_rew = 10.0, gamma = 0.99, eps = 1e-8;
    hipStream_t stream = nullptr, own_stream = nullptr;
    double* d_stats = nullptr;   // [obs_mean D][obs_var D][obs_count][ret mean, var, count]
    double* d_returns = nullptr;
    double* d_ep_ret = nullptr;
    int* d_ep_len = nullptr;
    std::string err;
    double* obs_mean() { return d_stats; }
    double* obs_var() { return d_stats + obs_dim; }
    double* obs_count() { return d_stats + 2 * obs_dim; }
    double* ret_stats() { return d_stats + 2 * obs_dim + 1; }
    int n_stats() const { return 2 * obs_dim + 4; }
};

#define NCHK(n, expr)                                                      \
    do {                                                                   \
        hipError_t _e = (expr);                                            \
        if (_e != hipSuccess) {                                            \
            (n)->err = std::string(#expr) + ": " + hipGetErrorString(_e);  \
            return MRP_E_HIP;                                              \
        }                                                                  \
    } while (0)

extern "C" {

const char* mrp_norm_last_error(const mrp_norm* n) { return n ? n->err.c_str() : g_norm_create_error.c_str(); }

void mrp_norm_destroy(mrp_norm* n) {
    if (!n) return;
    (void)hipSetDevice(n->device);
    if (n->stream) (void)hipStreamSynchronize(n->stream);
    void* bufs[] = {n->d_stats, n->d_returns, n->d_ep_ret, n->d_ep_len};
    for (void* p : bufs)
        if (p) (void)hipFree(p);
    if (n->own_stream) (void)hipStreamDestroy(n->own_stream);
    delete n;
}

int mrp_norm_create(int n_lanes, int obs_dim, int device, double clip_obs, double clip_reward, double gamma, double epsilon,
                    mrp_norm** out) {
    g_norm_create_error.clear();
    if (!out || n_lanes <= 0 || obs_dim <= 0) { g_norm_create_error = "bad argument"; return MRP_E_ARG; }
    *out = nullptr;
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0) {
        g_norm_create_error = "no HIP device available (no CPU fallback)";
        return MRP_E_HIP;
    }
    if (device < 0 || device >= ndev) { g_norm_create_error = "device index out of range"; return MRP_E_ARG; }
    mrp_norm* n = new (std::nothrow) mrp_norm();
    if (!n) { g_norm_create_error = "out of host memory"; return MRP_E_ARG; }
    n->n_lanes = n_lanes; n->obs_dim = obs_dim; n->device = device;
    n->clip_obs = clip_obs; n->clip_rew = clip_reward; n->gamma = gamma; n->eps = epsilon;
    auto fail = [&](const char* what, hipError_t e) {
        g_norm_create_error = std::string(what) + ": " + hipGetErrorString(e);
        mrp_norm_destroy(n);
        return MRP_E_HIP;
    };
    hipError_t e;
    if ((e = hipSetDevice(device)) != hipSuccess) return fail("hipSetDevice", e);
    if ((e = hipStreamCreateWithFlags(&n->own_stream, hipStreamNonBlocking)) != hipSuccess) return fail("hipStreamCreate", e);
    n->stream = n->own_stream;
    size_t L = (size_t)n_lanes;
    if ((e = hipMalloc(&n->d_stats, n->n_stats() * sizeof(double))) != hipSuccess) return fail("hipMalloc", e);
    if ((e = hipMalloc(&n->d_returns, L * sizeof(double))) != hipSuccess) return fail("hipMalloc", e);
    if ((e = hipMalloc(&n->d_ep_ret, L * sizeof(double))) != hipSuccess) return fail("hipMalloc", e);
    if ((e = hipMalloc(&n->d_ep_len, L * sizeof(int))) != hipSuccess) return fail("hipMalloc", e);
    // RunningMeanStd(epsilon=1e-4): mean 0, var 1, count 1e-4 (obs and returns)
    double* h = new double[n->n_stats()];
    for (int j = 0; j < obs_dim; ++j) { h[j] = 0.0; h[obs_dim + j] = 1.0; }
    h[2 * obs_dim] = 1e-4;
    h[2 * obs_dim + 1] = 0.0; h[2 * obs_dim + 2] = 1.0; h[2 * obs_dim + 3] = 1e-4;
    e = hipMemcpy(n->d_stats, h, n->n_stats() * sizeof(double), hipMemcpyHostToDevice);
    delete[] h;
    if (e != hipSuccess) return fail("hipMemcpy", e);
    if ((e = hipMemset(n->d_returns, 0, L * sizeof(double))) != hipSuccess) return fail("hipMemset", e);
    if ((e = hipMemset(n->d_ep_ret, 0, L * sizeof(double))) != hipSuccess) return fail("hipMemset", e);
    if ((e = hipMemset(n->d_ep_len, 0, L * sizeof(int))) != hipSuccess) return fail("hipMemset", e);
    *out = n;
    return MRP_OK;
}

int mrp_norm_set_stream(mrp_norm* n, void* hip_stream) {
    if (!n) return MRP_E_ARG;
    n->stream = (hipStream_t)hip_stream;   // NULL: the HIP null stream (torch's default stream)
    return MRP_OK;
}

int mrp_norm_set_training(mrp_norm* n, int training) {
    if (!n) return MRP_E_ARG;
    n->training = training ? 1 : 0;
    return MRP_OK;
}

int mrp_norm_set_norm_obs(mrp_norm* n, int norm_obs) {
    if (!n) return MRP_E_ARG;
    n->norm_obs = norm_obs ? 1 : 0;
    return MRP_OK;
}

static int norm_launch(mrp_norm* n, const float* obs, const float* reward, const double* reward64, const uint8_t* done,
                       const float* term, float* obs_out, float* reward_out, float* term_out, double* ep_ret_out, int* ep_len_out, int step) {
    NCHK(n, hipSetDevice(n->device));
    const int L = n->n_lanes, D = n->obs_dim;
    // SB3 VecNormalize: obs statistics move when training and norm_obs, the returns' when training
    const int upd_obs = n->training && n->norm_obs, upd_ret = step && n->training;
    if (upd_obs || upd_ret) {
        hipLaunchKernelGGL(k_moments, dim3(D + 1), dim3(NT), 0, n->stream, obs, L, D, reward, n->d_returns, n->gamma,
                           n->obs_mean(), n->obs_var(), n->obs_count(), n->ret_stats(), upd_obs, upd_ret);
        NCHK(n, hipGetLastError());
    }
    const int nthreads = L * D > L ? L * D : L;
    hipLaunchKernelGGL(k_apply, dim3((nthreads + NT - 1) / NT), dim3(NT), 0, n->stream, obs, term, L, D, n->obs_mean(),
                       n->obs_var(), n->obs_count(), upd_obs, n->ret_stats(), n->clip_obs, n->clip_rew, n->eps, reward, reward64,
                       done, n->d_returns, obs_out, term_out, reward_out, n->d_ep_ret, n->d_ep_len, ep_ret_out, ep_len_out, step);
    NCHK(n, hipGetLastError());
    return MRP_OK;
}

int mrp_norm_reset_device(mrp_norm* n, const float* d_obs, float* d_obs_out) {
    if (!n || !d_obs || !d_obs_out) return MRP_E_ARG;
    return norm_launch(n, d_obs, nullptr, nullptr, nullptr, nullptr, d_obs_out, nullptr, nullptr, nullptr, nullptr, 0);
}

int mrp_norm_step_device_ex(mrp_norm* n, const float* d_obs, const float* d_reward, const double* d_reward64, const uint8_t* d_done,
                            const float* d_term_obs, float* d_obs_out, float* d_reward_out, float* d_term_out, double* d_ep_return,
                            int32_t* d_ep_len) {
    if (!n || !d_obs || !d_reward || !d_done || !d_obs_out || !d_reward_out) return MRP_E_ARG;
    return norm_launch(n, d_obs, d_reward, d_reward64, d_done, d_term_obs, d_obs_out, d_reward_out, d_term_out, d_ep_return,
                       d_ep_len, 1);
}

int mrp_norm_step_device(mrp_norm* n, const float* d_obs, const float* d_reward, const uint8_t* d_done, const float* d_term_obs,
                         float* d_obs_out, float* d_reward_out, float* d_term_out, double* d_ep_return, int32_t* d_ep_len) {
    return mrp_norm_step_device_ex(n, d_obs, d_reward, nullptr, d_done, d_term_obs, d_obs_out, d_reward_out, d_term_out,
                                   d_ep_return, d_ep_len);
}

int mrp_norm_get_stats(mrp_norm* n, double* out) {
    if (!n || !out) return MRP_E_ARG;
    NCHK(n, hipSetDevice(n->device));
    NCHK(n, hipMemcpyAsync(out, n->d_stats, n->n_stats() * sizeof(double), hipMemcpyDeviceToHost, n->stream));
    NCHK(n, hipStreamSynchronize(n->stream));
    return MRP_OK;
}

int mrp_norm_set_stats(mrp_norm* n, const double* in) {
    if (!n || !in) return MRP_E_ARG;
    NCHK(n, hipSetDevice(n->device));
    NCHK(n, hipMemcpyAsync(n->d_stats, in, n->n_stats() * sizeof(double), hipMemcpyHostToDevice, n->stream));
    NCHK(n, hipStreamSynchronize(n->stream));
    return MRP_OK;
}

}  // extern "C"
