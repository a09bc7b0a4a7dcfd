/*
 * mrp.h -- C ABI of the MI355X-native MultiRobotPuzzle step library (libmrp.so).
 *
 * Drop-in boundary for the gym_puzzles hot path.  In the reference the per-step work is
 * Python driving pybox2d object-by-object (~20 SWIG crossings per agent per step plus
 * C++->Python contact callbacks); here one call advances N independent worlds ("lanes")
 * on one GPU.  Each entry point names the reference interface it replaces.
 *
 * Conventions
 *   - Plain C types only; all arrays are row-major [n_lanes][dim].
 *   - Functions return 0 on success, a negative MRP_E* code on failure; mrp_last_error()
 *     gives the message (per context, or the last create failure when ctx == NULL).
 *   - "_device" variants take device pointers (hipMalloc / torch.cuda tensors) and are
 *     asynchronous on the context's stream; the plain variants take host pointers and
 *     synchronize.
 *   - Not re-entrant per context; one context per (device, stream, thread).
 *
 * env_id:  0 MultiRobotPuzzle-v0       (gym_puzzles/__init__.py:3-8,  multi_robot_puzzle_00.py:142)
 *          1 MultiRobotPuzzleHeavy-v0  (gym_puzzles/__init__.py:10-15, multi_robot_puzzle_00.py:606)
 *          2 MultiRobotPuzzle-v2       (gym_puzzles/__init__.py:17-22, multi_robot_puzzle_02.py:126)
 *          3 MultiRobotPuzzleHeavy-v2  (gym_puzzles/__init__.py:24-29, multi_robot_puzzle_02.py:711)
 *          4 MultiRobotPuzzleHeavy-v2 with the build-defined 3-block square
 *          5 MultiRobotPuzzle-v3       (gym_puzzles/__init__.py:31-35, core.py:77 RobotPuzzleBase)
 *          6 MultiRobotPuzzle-v3 constructed with heavy=True (gym_puzzles/tests/test_env.py:12)
 *          7-10  MultiRobotPuzzle2(num_agents=1, 3, 4, 5)      (multi_robot_puzzle_02.py:139,151,354)
 *          11-14 MultiRobotPuzzleHeavy2(num_agents=1, 3, 4, 5) (multi_robot_puzzle_02.py:711)
 *          15-18 RobotPuzzleBase(num_agents=1, 3, 4, 5)        (core.py:86-106,230)
 *          19-22 RobotPuzzleBase(num_agents=1, 3, 4, 5, heavy=True)
 */
#ifndef MRP_H
#define MRP_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define MRP_OK 0
#define MRP_E_ARG (-1)     /* bad argument (env id, lane count, null pointer) */
#define MRP_E_HIP (-2)     /* HIP runtime error (no device, launch failure, OOM) */
#define MRP_E_STATE (-3)   /* call order violation (e.g. step before reset) */

/* lane status codes written by mrp_step (the reference's done_status strings) */
#define MRP_STATUS_RUNNING 0
#define MRP_STATUS_PUZZLE_COMPLETE 1   /* multi_robot_puzzle_00.py:515-519, _02.py:575-582 */
#define MRP_STATUS_AGENT_OOB 2         /* multi_robot_puzzle_02.py:552-556 */
#define MRP_STATUS_BLOCK_OOB 3         /* multi_robot_puzzle_02.py:558-562 */
/* flag bits OR-ed into the status byte (SURVEY.md 8b "Errors": per-lane NaN is reported, never a
 * crash; the reference would carry the NaN on silently, multi_robot_puzzle_00.py:521 returns {}) */
#define MRP_STATUS_KIND_MASK 0x3f
#define MRP_STATUS_NONFINITE 0x40      /* this step's observation or a dynamic body's state holds NaN/inf */
#define MRP_STATUS_FAULT 0x80          /* a loop guard has tripped in this lane (sticky; code: mrp_get_faults) */

typedef struct mrp_ctx mrp_ctx;

/* Static dimensions of an env id: observation_space / action_space shapes
 * (multi_robot_puzzle_00.py:186-207, _02.py:174-195), number of spawn draws per reset,
 * agents, blocks and the TimeLimit max_episode_steps (gym_puzzles/__init__.py:6-27).
 * MRP_E_STATE if the library's compiled layout of the env disagrees with its tables (a build defect). */
int mrp_env_dims(int env_id, int* obs_dim, int* act_dim, int* n_draws, int* n_agents, int* n_blocks,
                 int* max_episode_steps);

/* Create n_lanes worlds on HIP device `device`.  Replaces gym.make(id) ->
 * MultiRobotPuzzle.__init__ (multi_robot_puzzle_00.py:152-209): one Box2D.b2World per lane
 * (gravity 0, no sleep).  `seed` keys the on-device counter RNG (device resets, synthetic
 * actions); `lane_offset` is the global index of lane 0 (multi-GPU sharding keeps per-lane
 * streams identical for any GPU count).  Worlds are empty until mrp_reset. */
int mrp_create(int env_id, int n_lanes, int device, uint64_t seed, uint64_t lane_offset, mrp_ctx** out);
void mrp_destroy(mrp_ctx* ctx);
const char* mrp_last_error(const mrp_ctx* ctx);
int mrp_n_lanes(const mrp_ctx* ctx);
int mrp_env_id(const mrp_ctx* ctx);

/* Use this hipStream_t for all subsequent work; NULL selects the HIP null stream (torch's default
 * stream, cuda_stream == 0).  A new context runs on its own non-blocking stream until this is called. */
int mrp_set_stream(mrp_ctx* ctx, void* hip_stream);
int mrp_synchronize(mrp_ctx* ctx);

/* set_reward_params (multi_robot_puzzle_00.py:231-239, _02.py:216-225; v3 core.py:149-155, where
 * puzzle_comp is the completion bonus step() adds unshaped and the two penalties are unused). */
int mrp_set_reward_params(mrp_ctx* ctx, double agent_delta, double agent_distance, double block_delta,
                          double block_distance, double puzzle_comp, double out_of_bounds, double blk_out_of_bounds);
/* update_params(timestep, decay) (multi_robot_puzzle_00.py:241-243, _02.py:227-230; v3 stores a value
 * its step() never reads, core.py:158-159, so it changes nothing there). */
int mrp_update_params(mrp_ctx* ctx, double timestep, double decay);
/* update_goal(epoch, nb_epochs) (multi_robot_puzzle_00.py:245-246, _02.py:232-233). */
int mrp_update_goal(mrp_ctx* ctx, double epoch, double nb_epochs);

/* reset() (multi_robot_puzzle_00.py:392-411, _02.py:421-442) for the lanes whose
 * lane_mask byte is nonzero (NULL = all): destroy + rebuild the bodies in the reference's
 * order, then the reference's extra physics step with a random action.
 *   draws   [n_lanes][n_draws] float64: the np.random.uniform(...) values the reference
 *           draws (gym_puzzles_amd/spawn.py); NULL = device counter RNG.
 *   actions [n_lanes][act_dim] float32: the reset step's action_space.sample(); NULL = RNG.
 *   obs     [n_lanes][obs_dim] float32 out (rows of unmasked lanes are left untouched). */
int mrp_reset(mrp_ctx* ctx, const uint8_t* lane_mask, const double* draws, const float* actions, float* obs);
int mrp_reset_device(mrp_ctx* ctx, const uint8_t* d_lane_mask, const double* d_draws, const float* d_actions,
                     float* d_obs);

/* step(action) (multi_robot_puzzle_00.py:413-521, _02.py:444-584) under gym's TimeLimit
 * wrapper, for all lanes:
 *   actions  [n_lanes][act_dim] float32 (NULL = device RNG uniform[-1,1), keyed by lane/step)
 *   obs      [n_lanes][obs_dim] float32 out (the reference returns float64; values are
 *            float32(reference value))
 *   reward   [n_lanes] float32 out, done/truncated [n_lanes] uint8 out
 *            (truncated = TimeLimit.truncated), status [n_lanes] uint8 out (MRP_STATUS_*),
 *   terminal_obs [n_lanes][obs_dim] float32 out or NULL: when auto-reset is on, done lanes
 *            are reset on device (RNG spawns) and obs holds the new episode's first
 *            observation while terminal_obs holds the last one (SB3 VecEnv semantics).
 * Any output pointer except obs may be NULL. */
int mrp_step(mrp_ctx* ctx, const float* actions, float* obs, float* reward, uint8_t* done, uint8_t* truncated,
             uint8_t* status, float* terminal_obs);
int mrp_step_device(mrp_ctx* ctx, const float* d_actions, float* d_obs, float* d_reward, uint8_t* d_done,
                    uint8_t* d_truncated, uint8_t* d_status, float* d_terminal_obs);
/* As mrp_step / mrp_step_device, plus `reward64` [n_lanes] float64 out (may be NULL): the reward
 * exactly as the reference returns it (a Python float, multi_robot_puzzle_00.py:521,
 * _02.py:584), before the float32 rounding of `reward`.  Monitor's episode return sums these. */
int mrp_step_ex(mrp_ctx* ctx, const float* actions, float* obs, float* reward, double* reward64, uint8_t* done,
                uint8_t* truncated, uint8_t* status, float* terminal_obs);
int mrp_step_device_ex(mrp_ctx* ctx, const float* d_actions, float* d_obs, float* d_reward, double* d_reward64,
                       uint8_t* d_done, uint8_t* d_truncated, uint8_t* d_status, float* d_terminal_obs);
/* n_steps consecutive step() calls of every lane in ONE launch (synthetic rollouts, evaluation
 * with device-RNG or pre-computed actions): the lane state stays on chip between the steps, and
 * each step writes its outputs exactly as one mrp_step_device_ex would (step s of lane l at row
 * s * n_lanes + l of every array: d_actions [n_steps][n_lanes][act_dim] or NULL = device RNG,
 * d_obs / d_terminal_obs [n_steps][n_lanes][obs_dim], the others [n_steps][n_lanes]).  The result
 * is bit-identical to n_steps single steps; lanes advance independently inside the launch. */
int mrp_step_n_device(mrp_ctx* ctx, int n_steps, const float* d_actions, float* d_obs, float* d_reward, double* d_reward64,
                      uint8_t* d_done, uint8_t* d_truncated, uint8_t* d_status, float* d_terminal_obs);
int mrp_set_auto_reset(mrp_ctx* ctx, int enabled);
/* frameskip: world.Step(1/50, 180, 60) calls per env step, 1-64 (default 1).  Replaces the
 * MultiRobotPuzzle2(frameskip=k) constructor argument (multi_robot_puzzle_02.py:139,146,476-478:
 * `for _ in range(self.frameskip): self.world.Step(...)`; the reset's extra step takes it too). */
int mrp_set_frameskip(mrp_ctx* ctx, int frameskip);
/* Re-key the device counter RNG (spawns of later resets, synthetic actions) without touching the
 * lanes, parameters, stream or time limit: SB3 VecEnv.seed(seed) (train/train.py:63-75 seeds
 * every env before the first reset).  Per-lane streams stay keyed by the global lane index. */
int mrp_set_seed(mrp_ctx* ctx, uint64_t seed);
/* Lane scheduling: with costliest_first = 1 each step dispatches the lanes in descending order of
 * their previous step's cost, so the long serial solver chains start first (one small sort kernel
 * per step); 0 keeps lane order.  Results never depend on it.  The default is per env id, set by
 * mrp_create: on for Heavy-v0 (env 1) and v3 (env 5) when n_lanes exceeds the lanes k_step keeps
 * resident at once (CUs x 4 SIMDs x its waves per SIMD), off otherwise (round-4 A/B, DESIGN.md:
 * Heavy-v0 +4 %, v3 +1-2 %; v0 -0.9 % at 4096 lanes and -3..-5 % at 1024). */
int mrp_set_schedule(mrp_ctx* ctx, int costliest_first);
/* the context's current lane scheduling mode (the per-env default until mrp_set_schedule) */
int mrp_get_schedule(const mrp_ctx* ctx);
/* TimeLimit max_episode_steps applied inside mrp_step (default: the registered value of
 * gym_puzzles/__init__.py:6-27); 0 disables it (when an outer gym.wrappers.TimeLimit is used). */
int mrp_set_time_limit(mrp_ctx* ctx, int max_episode_steps);

/* Introspection (tests, checkpointing).  Dynamic bodies in creation order (blocks, agents),
 * 6 floats each: worldCenter.x, worldCenter.y, angle, linearVelocity.x, .y, angularVelocity. */
int mrp_get_bodies(mrp_ctx* ctx, float* out /* [n_lanes][6*(n_blocks+n_agents)] */);
/* per lane: goal_contact flags [n_agents] then blks_in_place -> int32 [n_lanes][n_agents+1] */
int mrp_get_flags(mrp_ctx* ctx, int32_t* out);
/* per lane: 0, or the code of the loop guard that ended a runaway loop in that lane (a bound no
 * valid world reaches: tree walks, contact-list walks, islands, TOI passes; see mrp_world.h
 * MRP_FAULT_*: 1-8 loop guards -- tree walks, contact-list walks, islands, TOI passes, pair decoding,
 * island DFS; 9-12 pool guards -- tree nodes, contact slots, move buffer, island arrays).  Sticky.
 * int32 [n_lanes] */
int mrp_get_faults(mrp_ctx* ctx, int32_t* out);
/* summed over lanes: TOI events and position-solver iterations (diagnostics) */
int mrp_counters(mrp_ctx* ctx, int64_t* toi_events, int64_t* pos_iters);
/* per-batch counters (SURVEY.md 5 "Metrics"), summed over lanes since mrp_create, reduced on the
 * device: out[8] = steps, resets, TOI events, position iterations, touching contacts (after each
 * world.Step's Collide), lane-steps with a non-finite output, lanes with a tripped loop guard, 0 */
int mrp_counters_ex(mrp_ctx* ctx, int64_t* out8);
/* Raw per-lane state (checkpoint / resume): mrp_state_words() 32-bit words per lane. */
int mrp_state_words(int env_id);
int mrp_get_state(mrp_ctx* ctx, uint32_t* out /* [n_lanes][state_words] */);
int mrp_set_state(mrp_ctx* ctx, const uint32_t* in);

/* rgb_array rendering, replacing render(mode='rgb_array') of
 * gym_puzzles/envs/multi_robot_puzzle_00.py:528-592 and multi_robot_puzzle_02.py:590-661
 * (_render_human_vision).  Renders the n selected lanes into uint8 RGB images
 * [n][height][width][3], row 0 at the top (the reference's `arr[::-1]`, :598); the full-size
 * viewport is 640x480 (v0) / 1440x810 (v2), other sizes resample the same scene.  The
 * rasteriser is defined in gym_puzzles_amd/csrc/mrp_render.h.  _device: device pointers,
 * asynchronous on the ctx stream; plain: host pointers, synchronous. */
int mrp_render_device(mrp_ctx* ctx, const int32_t* d_lanes, int n, int width, int height, uint8_t* d_rgb);
int mrp_render(mrp_ctx* ctx, const int32_t* lanes, int n, int width, int height, uint8_t* rgb);
/* per lane block_final_pos (x, y, angle) per block, in the units of the reference's
 * block_final_pos (v0 px, v2 scaled units): double [n_lanes][n_blocks][3] */
int mrp_get_goals(mrp_ctx* ctx, double* out);
/* host-only: the env's fixture geometry (creation order; local vertices, 16 fixtures x 8
 * vertices x (x, y); unused entries 0 / fix_body -1) */
int mrp_shapes(int env_id, int32_t* n_fix, int32_t* fix_body, int32_t* counts, float* verts);

/* Device self-test of the glibc-faithful sinf/cosf of every b2Rot::Set on the GPU: evaluates
 * b2Rot::Set (sin, cos) as the step does on device `device` for n host inputs (host output arrays). */
int mrp_selftest_sincos(int device, const float* x, float* sin_out, float* cos_out, int n);
/* Diagnostic builds (-DMRP_STAMPS) only: per-phase cycle totals of thread 0 since the last call
 * (returns MRP_E_STATE in the shipped build). */
int mrp_debug_stamps(int device, uint64_t* out16);
/* Diagnostic builds only: per-phase maxima over lane-steps, the slowest lane's total per step
 * (256 slots, indexed by step counter mod 256) and the (s_memtime, s_memrealtime) sums of lane
 * totals since the last call. */
int mrp_debug_stamps_ext(int device, uint64_t* pmax16, uint64_t* stepmax256, uint64_t* rt2);
/* Diagnostic builds only: the last step's per-lane trace, n_lanes x MRP_TRACE_WORDS words (phase
 * cycles 0-10, total, island contacts, TOI events, position iterations, velocity-solver contact
 * units, velocity-sweep / position-pass / island set-up cycles, the TOI split (20-21), the collide
 * split (22-23), the lane timeline words (24-31), then the solve's thread-0 bookkeeping (32 island
 * building, 33 island write-back + integration, 34 fixture synchronisation) and the TOI scan alone (35)).  `out` must hold n_lanes * mrp_debug_trace_words()
 * words; it is left untouched (MRP_E_STATE) when the library has no diagnostic unit. */
#define MRP_TRACE_WORDS 40
int mrp_debug_trace_words(void);
int mrp_debug_trace(int device, uint32_t* out, int n_lanes);
/* Diagnostic builds (-DMRP_PROGRESS) only: allocate n_lanes host-mapped words that every lane's
 * thread 0 overwrites with the last progress point it reached; readable while a launch runs
 * (hang localisation).  Returns MRP_E_STATE in the shipped build. */
int mrp_debug_progress(int device, uint32_t** host_words, int n_lanes);
/* Diagnostic micro-benchmark: `blocks` workgroups each sweep a synthetic v0 island (nc agent-block
 * contacts of pcount points) `iters` times with the early exit off; cycles[block] = s_memtime
 * cycles of the sweeps (per-contact-update cost = cycles / (iters * nc)). */
int mrp_debug_velbench(int device, int nc, int pcount, int iters, int blocks, uint64_t* cycles);
/* Diagnostic micro-benchmark: `blocks` workgroups each run the position passes (up to `iters`) of a
 * synthetic island of nc static-wall contacts of pcount points squeezing one block (the passes never
 * reach the exit test); out[2 * block] = s_memtime cycles, out[2 * block + 1] = passes run. */
int mrp_debug_posbench(int device, int nc, int pcount, int iters, int blocks, uint64_t* out);

/* ------------------------------------------------------------------------------------------
 * On-device VecNormalize + Monitor statistics.  Replaces the host-side
 * stable-baselines3 wrappers the reference trains with: Monitor(env) per env
 * (train/train.py:68) and VecNormalize(DummyVecEnv(...)) with default arguments
 * (train/train.py:80-82; loaded back by train/test.py:66).  The statistics live on the device;
 * inputs and outputs are device arrays of a step's outputs ([n_lanes][obs_dim] float32 obs,
 * [n_lanes] float32 reward, uint8 done).  Asynchronous on the context's stream.
 * ------------------------------------------------------------------------------------------ */
typedef struct mrp_norm mrp_norm;

/* VecNormalize(clip_obs, clip_reward, gamma, epsilon); RunningMeanStd(epsilon=1e-4) for obs and returns */
int mrp_norm_create(int n_lanes, int obs_dim, int device, double clip_obs, double clip_reward, double gamma, double epsilon,
                    mrp_norm** out);
void mrp_norm_destroy(mrp_norm* n);
const char* mrp_norm_last_error(const mrp_norm* n);
int mrp_norm_set_stream(mrp_norm* n, void* hip_stream);   /* as mrp_set_stream: NULL = the HIP null stream */
/* VecNormalize.training: statistics update on (1) or frozen (0, evaluation) */
int mrp_norm_set_training(mrp_norm* n, int training);
/* VecNormalize.norm_obs: with 0 the observation statistics are not updated (SB3 updates obs_rms
 * only when training and norm_obs); the normalised outputs are still written */
int mrp_norm_set_norm_obs(mrp_norm* n, int norm_obs);
/* VecNormalize.reset: update obs statistics, normalise obs, zero the discounted returns and
 * the Monitor accumulators */
int mrp_norm_reset_device(mrp_norm* n, const float* d_obs, float* d_obs_out);
/* VecNormalize.step_wait + Monitor.step: normalised obs / reward (and terminal obs of done
 * lanes, optional), returns[done] = 0; for done lanes the finished episode's return (float64
 * sum of raw rewards) and length (Monitor's info["episode"] r / l; optional outputs) */
int mrp_norm_step_device(mrp_norm* n, const float* d_obs, const float* d_reward, const uint8_t* d_done, const float* d_term_obs,
                         float* d_obs_out, float* d_reward_out, float* d_term_out, double* d_ep_return, int32_t* d_ep_len);
/* As mrp_norm_step_device; with d_reward64 (mrp_step_device_ex's float64 rewards, may be NULL) the
 * Monitor episode return sums the env's float64 rewards, as SB3's Monitor does (train/train.py:68). */
int mrp_norm_step_device_ex(mrp_norm* n, const float* d_obs, const float* d_reward, const double* d_reward64,
                            const uint8_t* d_done, const float* d_term_obs, float* d_obs_out, float* d_reward_out,
                            float* d_term_out, double* d_ep_return, int32_t* d_ep_len);
/* statistics as float64[2*obs_dim + 4]: obs mean[obs_dim], obs var[obs_dim], obs count,
 * return mean, return var, return count (VecNormalize save/load) */
int mrp_norm_get_stats(mrp_norm* n, double* out);
int mrp_norm_set_stats(mrp_norm* n, const double* in);

#ifdef __cplusplus
}
#endif
#endif
