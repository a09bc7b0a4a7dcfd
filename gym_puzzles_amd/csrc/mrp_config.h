// mrp_config.h -- per-environment static tables (geometry, mass, spawn bounds) and the
// compile-time dimensions of each registered MultiRobotPuzzle id.
//
// Env ids follow include/mrp.h: 0 MultiRobotPuzzle-v0, 1 MultiRobotPuzzleHeavy-v0,
// 2 MultiRobotPuzzle-v2, 3 MultiRobotPuzzleHeavy-v2, 4 Heavy-v2 with the build-defined
// 3-block square, 5 MultiRobotPuzzle-v3 (RobotPuzzleBase,
// core.py), 6 v3 constructed with heavy=True (tests/test_env.py:12), 7-10 MultiRobotPuzzle2
// constructed with num_agents = 1, 3, 4, 5 and 11-14 MultiRobotPuzzleHeavy2 with the same
// agent counts (multi_robot_puzzle_02.py:139,151,354), 15-18 / 19-22 RobotPuzzleBase(num_agents =
// 1, 3, 4, 5) with heavy False / True (core.py:86-106).
#pragma once
#include "mrp_math.h"

namespace mrp {

// status byte flags next to the terminal kind (include/mrp.h MRP_STATUS_NONFINITE / MRP_STATUS_FAULT)
constexpr int MRP_STATUS_NONFINITE_BIT = 0x40, MRP_STATUS_FAULT_BIT = 0x80;

constexpr int MAX_POLY = 8;
constexpr int MAXBODY = 10;   // bodies: blocks + agents + 4 walls (max over configs: 1 + 5 + 4)
constexpr int MAXF = 24;      // fixtures (max over configs: v2 with 5 agents, 2 + 5 * 3 + 4 = 21)
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
// MultiRobotPuzzle2(num_agents = N) (multi_robot_puzzle_02.py:139): one T block (2 fixtures),
// N agents (body + 2 wheels), 4 walls; CMAX = fixture pairs on different bodies, not both static
template <int N> struct DimsV2 {
    static constexpr int DF = 2 + 3 * N;   // dynamic fixtures
    static constexpr int V = 2, NA = N, NB = 1, NF = DF + 4, CMAX = DF * (DF - 1) / 2 - 1 - 3 * N + 4 * DF,
                         OBS = 9 * N + 4 + 16 + 1, ACT = 2 * N, NDRAW = 1 + 2 * N + 2;
};
template <> struct Dims<7> : DimsV2<1> {};
template <> struct Dims<8> : DimsV2<3> {};
template <> struct Dims<9> : DimsV2<4> {};
template <> struct Dims<10> : DimsV2<5> {};
template <> struct Dims<11> : DimsV2<1> {};
template <> struct Dims<12> : DimsV2<3> {};
template <> struct Dims<13> : DimsV2<4> {};
template <> struct Dims<14> : DimsV2<5> {};
// RobotPuzzleBase(num_agents = N) (core.py:88,106,230): one T block (2 fixtures), N Robots (1 fixture), 4 walls
template <int N> struct DimsV3 {
    static constexpr int DF = 2 + N;
    static constexpr int V = 3, NA = N, NB = 1, NF = DF + 4, CMAX = DF * (DF - 1) / 2 - 1 + 4 * DF,
                         OBS = 4 * N + 3 + 16, ACT = 3 * N, NDRAW = 3 + 2 * N;
};
template <> struct Dims<15> : DimsV3<1> {};
template <> struct Dims<16> : DimsV3<3> {};
template <> struct Dims<17> : DimsV3<4> {};
template <> struct Dims<18> : DimsV3<5> {};
template <> struct Dims<19> : DimsV3<1> {};
template <> struct Dims<20> : DimsV3<3> {};
template <> struct Dims<21> : DimsV3<4> {};
template <> struct Dims<22> : DimsV3<5> {};
static_assert(DimsV2<2>::CMAX == Dims<2>::CMAX && DimsV2<2>::OBS == Dims<2>::OBS && DimsV2<2>::NF == Dims<2>::NF &&
              DimsV2<2>::NDRAW == Dims<2>::NDRAW, "DimsV2 restates the registered v2 layout");
static_assert(DimsV3<2>::CMAX == Dims<5>::CMAX && DimsV3<2>::OBS == Dims<5>::OBS && DimsV3<2>::NF == Dims<5>::NF &&
              DimsV3<2>::NDRAW == Dims<5>::NDRAW && DimsV3<2>::ACT == Dims<5>::ACT, "DimsV3 restates the v3 layout");
constexpr int N_ENVS = 23;

// Per env id: version (0 v0, 2 v2, 3 v3), agents, blocks, heavy block, registered TimeLimit.
struct EnvCfg { int version, n_agents, n_blocks, heavy, max_steps; };
constexpr EnvCfg ENV_CFG[N_ENVS] = {
    {0, 2, 1, 0, 2000}, {0, 5, 1, 1, 3000}, {2, 2, 1, 0, 2000}, {2, 2, 1, 1, 2000}, {2, 2, 3, 1, 2000},
    {3, 2, 1, 0, 1500}, {3, 2, 1, 1, 1500},
    {2, 1, 1, 0, 2000}, {2, 3, 1, 0, 2000}, {2, 4, 1, 0, 2000}, {2, 5, 1, 0, 2000},
    {2, 1, 1, 1, 2000}, {2, 3, 1, 1, 2000}, {2, 4, 1, 1, 2000}, {2, 5, 1, 1, 2000},
    {3, 1, 1, 0, 1500}, {3, 3, 1, 0, 1500}, {3, 4, 1, 0, 1500}, {3, 5, 1, 0, 1500},
    {3, 1, 1, 1, 1500}, {3, 3, 1, 1, 1500}, {3, 4, 1, 1, 1500}, {3, 5, 1, 1, 1500},
};

// Node pool of a lane's dynamic tree.  b2DynamicTree starts at 16 nodes and doubles only when
// all are live; a world holds at most 2 * proxies - 1 live nodes, so an env with <= 8 proxies
// never grows past 16 and its node ids (free-list order) never exceed 15.  A pool allocated at
// its final size with the free list in index order hands out the same ids as Box2D's doubling
// pool (the doubled part is appended to the free list in index order once the old part is full).
template <int ENV> constexpr int tree_n() {
    return 2 * Dims<ENV>::NF - 1 <= 16 ? 16 : (2 * Dims<ENV>::NF - 1 <= 32 ? 32 : 64);
}
// Move buffer: at most NF proxies are buffered between two UpdatePairs (every proxy after a
// reset's CreateProxy calls; a moved proxy at most once per Solve / TOI sub-step)
template <int ENV> constexpr int move_n() { return Dims<ENV>::NF < 16 ? 16 : 32; }

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
