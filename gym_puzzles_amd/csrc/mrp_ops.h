// mrp_ops.h -- the per-env launch table between the C ABI (mrp_kernels.hip) and the per-env
// kernel translation units (mrp_env0.hip .. mrp_env6.hip).
//
// Every env id is its own template instantiation of the whole lane step (k_step<ENV> and
// friends), and each instantiation is compiled in its own translation unit so the seven
// builds run in parallel (build.py).  A translation unit exports one EnvOps: plain host
// functions that launch its kernels on a given stream.  The C ABI never names a kernel.
#pragma once
#include <hip/hip_runtime.h>

#include <cstddef>
#include <cstdint>

#include "mrp_config.h"

namespace mrpr {
struct RenderArgs {
    float sx, sy;              // world units per pixel
    float lw_unit;             // world units per viewport pixel (line widths)
    float ring_r;              // v2: scaled_epsilon / RATIO
    double goal_scale;         // lane goal units -> world metres
};
constexpr int RBLOCK = 256;
constexpr int RPPT = 8;        // pixels per thread: one display-list build serves RBLOCK*RPPT pixels
}  // namespace mrpr

namespace mrp {

constexpr int BLOCK = 64;      // one wave per workgroup: lanes of a block never wait on each other

// k_step's arguments (mrp_step_device_ex)
struct StepArgs {
    uint32_t* state;
    int nl;
    const float* actions;      // NULL: device RNG
    float* obs;
    float* reward;
    double* reward64;
    uint8_t* done;
    uint8_t* trunc;
    uint8_t* status;
    float* term_obs;
    EnvParams P;
    uint64_t seed, lane_offset;
    int auto_reset, max_steps;
    const int* order;          // NULL: workgroup b steps lane b
    uint32_t* cost;            // NULL: no per-lane cycle record
    const uint32_t* costmax;   // NULL: no cost-derived priority
    int nsteps;                // env steps per launch (mrp_step_n_device); step s of lane l writes row s * nl + l
};

// per-lane counters summed over the lanes (mrp_counters_ex), in this order
enum : int { CTR_STEPS = 0, CTR_RESETS, CTR_TOI, CTR_POS_ITERS, CTR_TOUCHING, CTR_NONFINITE, CTR_FAULT_LANES, CTR_N = 8 };

// diagnostic symbols of a -DMRP_STAMPS / -DMRP_PROGRESS build (debug_read's `what`)
enum : int { DBG_STAMPS = 0, DBG_PMAX = 1, DBG_STEPMAX = 2, DBG_RT = 3, DBG_TRACE = 4 };

struct EnvOps {
    int words;                 // lane_words<ENV>()
    int counters_word;         // word offset of LaneState::toiEvents (followed by posIters)
    int dims[6];               // Dims<ENV>: OBS, ACT, NDRAW, NA, NB, NF (mrp_create checks them against the tables)
    // contact-slot layout of LaneState (mrp_set_state repairs an understated high-water mark cHW):
    // word offset of cnext (the first of `cslot_arrays` contiguous arrays of `cslot_n` words) and of cHW
    int cslot_word, cslot_n, cslot_arrays, chw_word;
    int step_waves_per_eu;     // k_step's launch bound: resident waves per SIMD (mrp_create: resident lanes)
    hipError_t (*upload_tables)(const EnvTables* all);   // all N_ENVS tables -> this unit's __constant__ copy
    void (*init)(hipStream_t, uint32_t* state, int nl);
    void (*reset)(hipStream_t, uint32_t* state, int nl, const uint8_t* mask, const double* draws, const float* actions,
                  float* obs, const EnvParams& P, uint64_t seed, uint64_t lane_offset);
    void (*step)(hipStream_t, const StepArgs& a);
    void (*bodies)(hipStream_t, const uint32_t* state, int nl, float* out, int32_t* flags);
    void (*faults)(hipStream_t, const uint32_t* state, int nl, int32_t* out);
    void (*counters)(hipStream_t, const uint32_t* state, int nl, int64_t* out /* [CTR_N] */);
    void (*render)(hipStream_t, dim3 grid, const uint32_t* state, const int32_t* lanes, int nl, int W, int H,
                   const mrpr::RenderArgs& A, uint8_t* rgb);
    void (*goals)(hipStream_t, const uint32_t* state, int nl, double* out);
    // diagnostic builds only (MRP_E_STATE-like hipErrorNotSupported otherwise): copy `bytes` of
    // symbol `what` into `out` and zero it; point the progress word array at `dev_words`
    hipError_t (*debug_read)(int what, void* out, size_t bytes);
    hipError_t (*debug_progress)(uint32_t* dev_words);
};

// defined in mrp_env<E>.hip
extern const EnvOps g_env_ops_0, g_env_ops_1, g_env_ops_2, g_env_ops_3, g_env_ops_4, g_env_ops_5, g_env_ops_6,
    g_env_ops_7, g_env_ops_8, g_env_ops_9, g_env_ops_10, g_env_ops_11, g_env_ops_12, g_env_ops_13, g_env_ops_14,
    g_env_ops_15, g_env_ops_16, g_env_ops_17, g_env_ops_18, g_env_ops_19, g_env_ops_20, g_env_ops_21, g_env_ops_22;
// defined in mrp_env0.hip: the lane-distributed velocity-sweep micro-benchmark (mrp_debug_velbench)
hipError_t velbench_launch(const EnvTables* all, int nc, int pcount, int iters, int blocks, unsigned long long* d_out);
// defined in mrp_env0.hip: the position-pass micro-benchmark (mrp_debug_posbench)
hipError_t posbench_launch(const EnvTables* all, int nc, int pcount, int iters, int blocks, unsigned long long* d_out);

inline const EnvOps* env_ops(int env_id) {
    static const EnvOps* const t[N_ENVS] = {&g_env_ops_0,  &g_env_ops_1,  &g_env_ops_2,  &g_env_ops_3,  &g_env_ops_4,
                                            &g_env_ops_5,  &g_env_ops_6,  &g_env_ops_7,  &g_env_ops_8,  &g_env_ops_9,
                                            &g_env_ops_10, &g_env_ops_11, &g_env_ops_12, &g_env_ops_13, &g_env_ops_14,
                                            &g_env_ops_15, &g_env_ops_16, &g_env_ops_17, &g_env_ops_18, &g_env_ops_19,
                                            &g_env_ops_20, &g_env_ops_21, &g_env_ops_22};
    return env_id >= 0 && env_id < N_ENVS ? t[env_id] : nullptr;
}

}  // namespace mrp
