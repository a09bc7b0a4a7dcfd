// mrp_config.h -- per-environment static tables (geometry, mass, spawn bounds) and the
// compile-time dimensions of each registered MultiRobotPuzzle id.
//
// Env ids follow include/mrp.h: 0 MultiRobotPuzzle-v0, 1 MultiRobotPuzzleHeavy-v0,
// 2 MultiRobotPuzzle-v2, 3 MultiRobotPuzzleHeavy-v2, 4 Heavy-v2 with the build-defined
// 3-block square, 5 MultiRobotPuzzle-v3 (RobotPuzzleBase,
// core.py), 6 v3 constructed with heavy=True (tests/test_env.py:12).
#pragma once
#include "mrp_math.h"

namespace mrp {

// status byte flags next to the terminal kind (include/mrp.h MRP_STATUS_NONFINITE / MRP_STATUS_FAULT)
constexpr int MRP_STATUS_NONFINITE_BIT = 0x40, MRP_STATUS_FAULT_BIT = 0x80;

constexpr int MAX_POLY = 8;
constexpr int TREE_N = 32;    // largest dynamic-tree node pool (15 proxies in the 3-block config)
constexpr int MOVE_N = 16;    // move buffer: at most NF (<= 15) proxies move between two UpdatePairs
constexpr int MAXB = 9;       // bodies: <= 3 blocks + 5 agents ... + 4 walls (max over configs: 1 + 5 + 4 = 10)
constexpr int MAXBODY = 10;
constexpr int MAXF = 16;
constexpr int MAXV = 16;
constexpr int MAXDRAW = 16;

// Compile-time dimensions per env id.  CMAX = fixture pairs on different bodies with at
// least one dynamic body (upper bound on live contacts).
template <int ENV> struct Dims;
template <> struct Dims<0> { static constexpr int V = 0, NA = 2, NB = 1, NF = 8, CMAX = 21, OBS = 28, ACT = 6, NDRAW = 7; };
template <> struct Dims<1> { static constexpr int V = 0, NA = 5, NB = 1, NF = 11, CMAX = 48, OBS = 40, ACT = 15, NDRAW = 13; };
template <> struct Dims<2> { static constexpr int V = 2, NA = 2, NB = 1, NF = 12, CMAX = 53, OBS = 39, ACT = 4, NDRAW = 7; };
template <> struct Dims<3> { static constexpr int V = 2, NA = 2, NB = 1, NF = 12, CMAX = 53, OBS = 39, ACT = 4, NDRAW = 7; };
template <> struct Dims<4> { static constexpr int V = 2, NA = 2, NB = 3, NF = 15, CMAX = 91, OBS = 69, ACT = 4, NDRAW = 9; };
template <> struct Dims<5> { static constexpr int V = 3, NA = 2, NB = 1, NF = 8, CMAX = 21, OBS = 27, ACT = 6, NDRAW = 7; };
template <> struct Dims<6> { static constexpr int V = 3, NA = 2, NB = 1, NF = 8, CMAX = 21, OBS = 27, ACT = 6, NDRAW = 7; };
constexpr int N_ENVS = 7;

// Node pool of a lane's dynamic tree.  b2DynamicTree starts at 16 nodes and doubles only when
// all are live; a world holds at most 2 * proxies - 1 live nodes, so an env with <= 8 proxies
// never grows past 16 and its node ids (free-list order) never exceed 15.
template <int ENV> constexpr int tree_n() { return 2 * Dims<ENV>::NF - 1 <= 16 ? 16 : 32; }

struct ShapeDef {
    int count;
    float radius;
    V2 v[MAX_POLY];
    V2 n[MAX_POLY];
};

// Body order everywhere: creation order of the reference = blocks, agents, walls.
struct EnvTables {
    int env_id, version, n_agents, n_blocks, n_dyn, n_bodies, n_fix, obs_dim, act_dim, n_draws, max_steps, pad;
    float mass[MAXBODY], invMass[MAXBODY], I[MAXBODY], invI[MAXBODY], lcx[MAXBODY], lcy[MAXBODY];
    float linDamp[MAXBODY], angDamp[MAXBODY];
    int body_fix0[MAXBODY], body_nfix[MAXBODY];
    int body_reset_mass[MAXBODY];      // 1 if any fixture had density > 0 (ResetMassData ran)
    float wall_px[4], wall_py[4];
    int fix_body[MAXF];
    float fix_friction[MAXF], fix_restitution[MAXF];
    ShapeDef shape[MAXF];
    int nverts[3];
    V2 verts[3][MAXV];
    double draw_lo[MAXDRAW], draw_hi[MAXDRAW];
    double block_px[3], block_py[3];   // v2: fixed spawn position per block
    float agent_angle;
    float pad2;
    double goal_x, goal_y, goal_a;     // v0 block_final_pos['t_block']
    double goal_off[3][3];             // 3-block: goal offsets (world m) + angle per block
};

// Reward / shaping parameters (set_reward_params, update_params, update_goal).
struct EnvParams {
    double w_dAgent, w_agentDist, w_dBlock, w_blkDist;
    double shaped_bounds, shaped_blk_bounds, shaped_puzzle;
    double scaled_epsilon;
    double puzzle_complete;            // v3 puzzle_complete_reward (core.py:155), added as is on completion
    int frameskip;                     // world.Step calls per env step (multi_robot_puzzle_02.py:139,476-478)
    int pad;
};

}  // namespace mrp
