/*
 * mrp_oracle.h -- TEST INFRASTRUCTURE ONLY (parity oracle; never linked into the product).
 *
 * CPU restatement of one MultiRobotPuzzle environment (one "lane"): the gym_puzzles
 * env logic of gym_puzzles/envs/multi_robot_puzzle_00.py (v0, Heavy-v0) and
 * multi_robot_puzzle_02.py (v2, Heavy-v2), driving the Box2D restatement in
 * b2_oracle.c.  Python float64 semantics (numpy 1.x scalar promotion, CPython float
 * pow/mod) are reproduced for the env-level arithmetic; the engine runs in float32.
 *
 * Parity against pybox2d is UNPINNED (no pybox2d / gym in this image and no reference
 * fixture pins a step result; SURVEY.md sections 4 and 8c).
 */
#ifndef MRP_ORACLE_H
#define MRP_ORACLE_H
#include <stdint.h>
#ifdef __cplusplus
extern "C" {
#endif

typedef struct OrEnv OrEnv;

/* env ids (same numbering as include/mrp.h) */
int or_obs_dim(int env_id);
int or_act_dim(int env_id);
int or_n_draws(int env_id);
int or_n_agents(int env_id);
int or_n_blocks(int env_id);
int or_max_episode_steps(int env_id);

OrEnv* or_create(int env_id);
void or_destroy(OrEnv* e);
/* reset(): draws are the values np.random.uniform(...) returns, in reference draw order;
 * action is the float32 action_space.sample() the reference feeds to its reset step. */
void or_reset(OrEnv* e, const double* draws, const float* reset_action, double* obs_out);
/* step(): returns env done (not TimeLimit) and terminal kind
 * (0 none, 1 puzzle complete, 2 agent out of bounds, 3 block out of bounds). */
void or_step(OrEnv* e, const float* action, double* obs_out, double* reward, int* done, int* kind);
void or_set_shaped(OrEnv* e, double bounds_penalty, double blk_bounds_penalty, double puzzle_reward);
/* world.Step calls per env step (MultiRobotPuzzle2(frameskip=k), multi_robot_puzzle_02.py:139,476-478) */
void or_set_frameskip(OrEnv* e, int frameskip);
/* dynamic body state in creation order (blocks, then agents): c.x c.y a v.x v.y w */
int or_get_bodies(const OrEnv* e, float* out);
void or_get_flags(const OrEnv* e, int* goal_contact, int* blks_in_place);
int or_contact_count(const OrEnv* e);
void or_counters(const OrEnv* e, long* toi_events, long* pos_iters);
/* toi events, position iterations, touching contacts after each Step's Collide (summed) */
void or_counters_ex(const OrEnv* e, long* out3);
/* proxy ids of all fixtures in creation order (blocks, agents, walls) */
int or_proxy_ids(const OrEnv* e, int* out);
int or_body_mass(const OrEnv* e, int i, float* out4);
long or_batch_run(int env_id, int n_lanes, int steps, uint64_t seed, uint64_t lane_offset, const double* lo,
                  const double* hi, int max_steps, int threads, double* seconds, float* bodies, double* rsum,
                  int* resets);
/* or_batch_run with `skip` untimed steps first; *seconds and the return value cover only the
 * `steps` steps after them (the CPU baseline on the GPU line's window) */
long or_batch_run_window(int env_id, int n_lanes, int skip, int steps, uint64_t seed, uint64_t lane_offset, const double* lo,
                         const double* hi, int max_steps, int threads, double* seconds, float* bodies, double* rsum,
                         int* resets);
/* which solver variant this library was built as (checker / port / early-exit port; oracle/Makefile) */
const char* or_build_kind(void);

/* capacity high-water marks of one lane since creation: max live contacts, max tree node id,
 * max move-buffer fill, max island bodies / contacts, max TOI-island bodies / contacts, tree node
 * capacity (the device keeps fixed pools per lane; tests check these stay inside them) */
void or_capacity(const OrEnv* e, int* out8);
/* or_batch_run's workload, returning the capacity maxima over all lanes in caps8 */
long or_batch_capacity(int env_id, int n_lanes, int steps, uint64_t seed, const double* lo, const double* hi, int max_steps,
                       int threads, int* caps8);

/* work model (b2_oracle.h OrWork): 20 counters of one lane since creation */
void or_work(const OrEnv* e, long* out20);
/* or_batch_run's workload; work[step][lane][20] receives each launch's work per lane */
long or_batch_work(int env_id, int n_lanes, int steps, uint64_t seed, const double* lo, const double* hi, int max_steps,
                   int threads, long* work);

/* glibc-faithful math exported for tests */
float or_sinf(float x);
float or_cosf(float x);
void or_sincos_batch(const float* x, float* s, float* c, int n);   /* glibc sinf/cosf over an array */

/* counter-based RNG shared with the device path (integer SplitMix64 mix) */
double or_rng_u01(uint64_t seed, uint64_t lane, uint64_t stream, uint64_t counter);

#ifdef __cplusplus
}
#endif
#endif
