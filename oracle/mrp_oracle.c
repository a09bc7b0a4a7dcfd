/*
 * mrp_oracle.c -- TEST INFRASTRUCTURE ONLY.  CPU restatement of the MultiRobotPuzzle
 * env step/reset (see mrp_oracle.h).  Every function cites the reference lines it
 * restates.  Engine calls go to b2_oracle.c; sinf/cosf/pow are the platform libm
 * (glibc), exactly what pybox2d's C++ and CPython's float ops call.
 *
 * Parity vs pybox2d: UNPINNED (no fixture in the reference pins a step result).
 */
#include "mrp_oracle.h"
#include "b2_oracle.h"

#include <math.h>
#include <stdlib.h>
#include <string.h>

/* ---------------------------------------------------------------- Python float semantics */
/* libm pow through a volatile pointer: gcc folds pow(x, 2.0) into x * x after inlining, but CPython's
 * `x ** 2` is a real glibc pow call, which is not correctly rounded (<= 0.52 ulp) and differs from
 * x * x in the last bit for rare inputs (found by tests/test_v2_env_layer.py's restatement) */
static double (*volatile libm_pow)(double, double) = pow;
/* CPython float_pow (Objects/floatobject.c) special cases, then libm pow */
static double py_pow(double iv, double iw) {
    int negate = 0;
    if (iw == 0.0) return 1.0;
    if (isnan(iv)) return iv;
    if (isnan(iw)) return iv == 1.0 ? 1.0 : iw;
    if (iv == 0.0) return iw > 0.0 ? (fmod(iw, 2.0) == 1.0 ? iv : 0.0) : INFINITY;
    if (iv < 0.0) { iv = -iv; negate = (fmod(fabs(iw), 2.0) == 1.0); }
    if (iv == 1.0) return negate ? -1.0 : 1.0;
    double ix = libm_pow(iv, iw);
    return negate ? -ix : ix;
}
/* CPython float_rem / numpy npy_remainder: result carries the divisor's sign */
static double py_mod(double vx, double wx) {
    double mod = fmod(vx, wx);
    if (mod != 0.0) { if ((wx < 0) != (mod < 0)) mod += wx; }
    else mod = copysign(0.0, wx);
    return mod;
}
/* distance() multi_robot_puzzle_00.py:130-132 / multi_robot_puzzle_02.py:106-108 */
static double py_distance(double ax, double ay, double bx, double by) {
    double x = py_pow(ax - bx, 2.0), y = py_pow(ay - by, 2.0);
    return py_pow(x + y, 0.5);
}

float or_sinf(float x) { return sinf(x); }
float or_cosf(float x) { return cosf(x); }
void or_sincos_batch(const float* x, float* s, float* c, int n) { for (int i = 0; i < n; ++i) { s[i] = sinf(x[i]); c[i] = cosf(x[i]); } }

/* ---------------------------------------------------------------- counter RNG (device-reset path) */
static uint64_t splitmix64(uint64_t x) {
    x += 0x9E3779B97F4A7C15ULL;
    x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ULL;
    x = (x ^ (x >> 27)) * 0x94D049BB133111EBULL;
    return x ^ (x >> 31);
}
double or_rng_u01(uint64_t seed, uint64_t lane, uint64_t stream, uint64_t counter) {
    uint64_t h = splitmix64(seed ^ splitmix64(lane ^ splitmix64(stream ^ splitmix64(counter))));
    return (double)(h >> 11) * 0x1.0p-53;
}

/* ---------------------------------------------------------------- configs (BASELINE.json configs) */
typedef struct { int version, n_agents, n_blocks, heavy, obs_dim, act_dim, n_draws, max_steps; } Cfg;
#define N_CFGS 23
static const Cfg CFGS[N_CFGS] = {
    {0, 2, 1, 0, 28, 6, 7, 2000},   /* MultiRobotPuzzle-v0        __init__.py:3-8 */
    {0, 5, 1, 1, 40, 15, 13, 3000}, /* MultiRobotPuzzleHeavy-v0   __init__.py:10-15 */
    {2, 2, 1, 0, 39, 4, 7, 2000},   /* MultiRobotPuzzle-v2        __init__.py:17-22 */
    {2, 2, 1, 1, 39, 4, 7, 2000},   /* MultiRobotPuzzleHeavy-v2   __init__.py:24-29 */
    {2, 2, 3, 1, 69, 4, 9, 2000},   /* Heavy-v2, 3-block square (build-defined) */
    {3, 2, 1, 0, 27, 6, 7, 1500},   /* MultiRobotPuzzle-v3 (RobotPuzzleBase)  __init__.py:31-35 */
    {3, 2, 1, 1, 27, 6, 7, 1500},   /* MultiRobotPuzzle-v3 with heavy=True (tests/test_env.py:12) */
    /* MultiRobotPuzzle2(num_agents=N) / MultiRobotPuzzleHeavy2(num_agents=N), _02.py:139,151,178-194:
     * obs 9 N + 4 + 16 + 1, action 2 N, draws 1 + 2 N + 2 */
    {2, 1, 1, 0, 30, 2, 5, 2000}, {2, 3, 1, 0, 48, 6, 9, 2000}, {2, 4, 1, 0, 57, 8, 11, 2000}, {2, 5, 1, 0, 66, 10, 13, 2000},
    {2, 1, 1, 1, 30, 2, 5, 2000}, {2, 3, 1, 1, 48, 6, 9, 2000}, {2, 4, 1, 1, 57, 8, 11, 2000}, {2, 5, 1, 1, 66, 10, 13, 2000},
    /* RobotPuzzleBase(num_agents=N[, heavy=True]), core.py:86-136: obs 4 N + 3 + 16, action 3 N, draws 3 + 2 N */
    {3, 1, 1, 0, 23, 3, 5, 1500}, {3, 3, 1, 0, 31, 9, 9, 1500}, {3, 4, 1, 0, 35, 12, 11, 1500}, {3, 5, 1, 0, 39, 15, 13, 1500},
    {3, 1, 1, 1, 23, 3, 5, 1500}, {3, 3, 1, 1, 31, 9, 9, 1500}, {3, 4, 1, 1, 35, 12, 11, 1500}, {3, 5, 1, 1, 39, 15, 13, 1500},
};
static int valid(int id) { return id >= 0 && id < N_CFGS; }
int or_obs_dim(int id) { return valid(id) ? CFGS[id].obs_dim : -1; }
int or_act_dim(int id) { return valid(id) ? CFGS[id].act_dim : -1; }
int or_n_draws(int id) { return valid(id) ? CFGS[id].n_draws : -1; }
int or_n_agents(int id) { return valid(id) ? CFGS[id].n_agents : -1; }
int or_n_blocks(int id) { return valid(id) ? CFGS[id].n_blocks : -1; }
int or_max_episode_steps(int id) { return valid(id) ? CFGS[id].max_steps : -1; }

/* v0 constants multi_robot_puzzle_00.py:38-88 */
#define V0_SCALE 30.0
#define V0_VW 640
#define V0_VH 480
#define V0_BORDER 1.0
#define V0_FR 0.999
#define V0_DAMP 5.0
#define V0_DENSE 5.0
#define V0_EPSILON 25.0
#define V0_S 2.0
/* v2 constants multi_robot_puzzle_02.py:39-66 */
#define V2_SCALE 560.0
#define V2_VW 1440
#define V2_VH 810
#define V2_BORDER 0.3
#define V2_BOUNDS 0.1
#define V2_FR 0.01
#define V2_DAMP 5.0
#define V2_BLK_DENSE 1.56
#define V2_AGT_DENSE 17.3
#define V2_FORCE 0.75
#define V2_EPSILON 0.1

/* v3 constants core.py:16-36, robot.py:7-15, blocks.py:10-13 */
#define V3_SCALE 30.0
#define V3_VW 640
#define V3_VH 480
#define V3_BORDER 1.0
#define V3_BLK_FR 2.5
#define V3_DAMP 5.0
#define V3_DENSE 5.0
#define V3_EPSILON 25.0
#define V3_AGT_SCALE 8.0
#define V3_AGT_DENSE 5.0
#define V3_MAX_SPEED 5.0

static const double PY_PI = 3.141592653589793;

struct OrEnv {
    Cfg cfg; int id;
    World* world;
    Body* blocks[3]; Body* agents[5]; Body* walls[4];
    int have_bodies;
    int goal_contact[5]; int wall_contact;
    double agent_dist[5]; double block_distance[3];
    int blks_in_place, prev_blks_in_place;
    double goal[3][3];           /* block_final_pos per block: x, y, angle */
    int nverts[3]; V2 verts[3][16];
    int verts_init[3];
    double scaled_epsilon;
    double w_dAgent, w_agentDist, w_dBlock, w_blkDist;
    double shaped_bounds, shaped_blk_bounds, shaped_puzzle;
    double puzzle_complete;      /* v3 puzzle_complete_reward (core.py:155; step() adds it directly) */
    int frameskip;               /* world.Step calls per env step (multi_robot_puzzle_02.py:139,476-478) */
};

/* ContactDetector.BeginContact/EndContact: multi_robot_puzzle_00.py:92-111, _02.py:85-102.
 * Last event wins per agent; wall flag is written but never read by obs/reward. */
static void on_contact(OrEnv* e, Contact* c, int value) {
    if (e->cfg.version == 3) return;   /* core.py:46-61 tests `agent in [fixtureA.body, ...]` with Robot
                                          wrappers against b2Body objects: never true, flags stay False */
    Body* bA = c->fA->body; Body* bB = c->fB->body;
    Body* goal = e->blocks[0];
    for (int i = 0; i < e->cfg.n_agents; ++i) {
        Body* ag = e->agents[i];
        if (ag == bA || ag == bB) {
            if (goal == bA || goal == bB) e->goal_contact[i] = value;
            if (bA->tag >= 100 || bB->tag >= 100) e->wall_contact = value;
        }
    }
}
static void cb_begin(void* ctx, Contact* c) { on_contact((OrEnv*)ctx, c, 1); }
static void cb_end(void* ctx, Contact* c) { on_contact((OrEnv*)ctx, c, 0); }

OrEnv* or_create(int env_id) {
    if (!valid(env_id)) return NULL;
    OrEnv* e = (OrEnv*)calloc(1, sizeof(OrEnv));
    e->cfg = CFGS[env_id]; e->id = env_id;
    e->world = b2o_world_create();   /* Box2D.b2World(gravity=(0,0), doSleep=False) :164 / :149 */
    if (e->cfg.version == 0) {       /* set_reward_params defaults :231-239 */
        e->w_dAgent = 10; e->w_agentDist = 0.1; e->w_dBlock = 50; e->w_blkDist = 0.025;
        e->scaled_epsilon = V0_EPSILON;
        /* set_final_loc :115-128 with PUZZLE_REL_LOCATION :83-88 */
        e->goal[0][0] = (double)(V0_VW / 2) + 0.0 * V0_SCALE;
        e->goal[0][1] = (double)(V0_VH / 2) + 0.75 * V0_SCALE;
        e->goal[0][2] = 0.0;
    } else if (e->cfg.version == 3) {   /* core.py:149-155 set_reward_params defaults; goal core.py:277-281 */
        e->w_dAgent = 10; e->w_agentDist = 0.1; e->w_dBlock = 50; e->w_blkDist = 0.025;
        e->scaled_epsilon = V3_EPSILON;
        e->goal[0][0] = 5.0 / 6.0 * (double)V3_VW - 4.0 / 3.0 * V3_BORDER;
        e->goal[0][1] = (double)(V3_VH / 2);
        e->goal[0][2] = 0.0;
    } else {                         /* _02.py:216-225 */
        e->w_dAgent = 10; e->w_agentDist = 0.25; e->w_dBlock = 25; e->w_blkDist = 0.1;
        e->scaled_epsilon = V2_EPSILON;
    }
    /* shaped_* only exist after update_params() (_02.py:227-230); default = decay 1, t 0 */
    e->shaped_bounds = 1000.0; e->shaped_blk_bounds = 100.0; e->shaped_puzzle = 10000.0;
    e->puzzle_complete = 100.0;
    return e;
}

void or_set_shaped(OrEnv* e, double b, double bb, double p) { e->shaped_bounds = b; e->shaped_blk_bounds = bb; e->shaped_puzzle = p; }

void or_destroy(OrEnv* e) { if (!e) return; b2o_world_destroy(e->world); free(e); }

/* _destroy multi_robot_puzzle_00.py:218-229 / _02.py:203-214 */
static void env_destroy_bodies(OrEnv* e) {
    if (!e->have_bodies) return;
    b2o_set_listener(e->world, NULL, NULL, NULL);
    if (e->cfg.version == 3) {   /* core.py:246-262: boundary, goal block, agents */
        for (int i = 0; i < 4; ++i) b2o_destroy_body(e->world, e->walls[i]);
        for (int i = 0; i < e->cfg.n_blocks; ++i) b2o_destroy_body(e->world, e->blocks[i]);
        for (int i = 0; i < e->cfg.n_agents; ++i) b2o_destroy_body(e->world, e->agents[i]);
        e->have_bodies = 0;
        return;
    }
    for (int i = 0; i < e->cfg.n_blocks; ++i) b2o_destroy_body(e->world, e->blocks[i]);
    for (int i = 0; i < 4; ++i) b2o_destroy_body(e->world, e->walls[i]);
    for (int i = 0; i < e->cfg.n_agents; ++i) b2o_destroy_body(e->world, e->agents[i]);
    e->have_bodies = 0;
}

static void add_box_fixture(Body* b, float hx, float hy, float cx, float cy, float density, float friction, int tag) {
    Poly p; b2o_poly_box_oriented(&p, hx, hy, (V2){cx, cy}, 0.0f);
    FixtureDef fd = { &p, density, friction, 0.0f, tag };
    b2o_create_fixture(b, &fd);
}

/* "SAVE vertices data" multi_robot_puzzle_00.py:355-361 / _02.py:344-350: fixture-list order
 * (newest fixture first), duplicates skipped; the list persists across resets. */
static void save_vertices(OrEnv* e, int bi) {
    Body* b = e->blocks[bi];
    for (Fixture* f = b->fixtureList; f; f = f->next) {
        if (!e->verts_init[bi]) {          /* first time: the fixture's vertex list itself */
            for (int k = 0; k < f->shape.count; ++k) e->verts[bi][e->nverts[bi]++] = f->shape.v[k];
            e->verts_init[bi] = 1;
            continue;
        }
        int n0 = e->nverts[bi];            /* list comprehension sees the list before extend() */
        for (int k = 0; k < f->shape.count; ++k) {
            V2 v = f->shape.v[k];
            int found = 0;
            for (int j = 0; j < n0; ++j) if (e->verts[bi][j].x == v.x && e->verts[bi][j].y == v.y) { found = 1; break; }
            if (!found) e->verts[bi][e->nverts[bi]++] = v;
        }
    }
}

static void gen_v0(OrEnv* e, const double* d) {
    int heavy = e->cfg.heavy;
    double scaled = heavy ? V0_S / 2 : V0_S;          /* :303-308 */
    double blk_dense = heavy ? V0_DENSE * 2 : V0_DENSE;
    int k = 0;
    /* _generate_blocks :309-361 (single t_block) */
    {
        BodyDef bd = { BT_DYNAMIC, { (float)d[k], (float)d[k + 1] }, (float)d[k + 2], (float)V0_DAMP, (float)V0_DAMP, 0 };
        k += 3;
        Body* b = b2o_create_body(e->world, &bd);
        add_box_fixture(b, (float)(1 / scaled), (float)(1 / scaled), 0.0f, (float)(-1 / scaled), (float)blk_dense, (float)V0_FR, 0);
        add_box_fixture(b, (float)(3 / scaled), (float)(1 / scaled), 0.0f, (float)(1 / scaled), (float)blk_dense, (float)V0_FR, 1);
        e->blocks[0] = b;
        save_vertices(e, 0);
    }
    /* _generate_agents :363-378 */
    const double S = V0_S;
    V2 poly[8] = {
        { (float)(-0.5 / S), (float)(-1.5 / S) }, { (float)(0.5 / S), (float)(-1.5 / S) }, { (float)(1.5 / S), (float)(-0.5 / S) }, { (float)(1.5 / S), (float)(0.5 / S) },
        { (float)(0.5 / S), (float)(1.5 / S) }, { (float)(-0.5 / S), (float)(1.5 / S) }, { (float)(-1.5 / S), (float)(0.5 / S) }, { (float)(-1.5 / S), (float)(-0.5 / S) } };
    Poly ap; b2o_poly_set(&ap, poly, 8);
    for (int i = 0; i < e->cfg.n_agents; ++i) {
        BodyDef bd = { BT_DYNAMIC, { (float)d[k], (float)d[k + 1] }, 0.0f, (float)V0_DAMP, (float)V0_DAMP, 10 + i };
        k += 2;
        Body* b = b2o_create_body(e->world, &bd);
        FixtureDef fd = { &ap, 0.0f, 0.2f, 0.0f, 0 };   /* fixtureDef defaults: density 0, friction 0.2 */
        b2o_create_fixture(b, &fd);
        e->agents[i] = b; e->goal_contact[i] = 0;
    }
    /* _generate_boundary :260-275 */
    const double bx[4] = { 0, 1, 0.5, 0.5 }, by[4] = { 0.5, 0.5, 0, 1 };
    for (int i = 0; i < 4; ++i) {
        double hx = i < 2 ? 1.0 : (double)V0_VW / V0_SCALE;
        double hy = i < 2 ? (double)V0_VH / V0_SCALE : 1.0;
        BodyDef bd = { BT_STATIC, { (float)((double)V0_VW / V0_SCALE * bx[i]), (float)((double)V0_VH / V0_SCALE * by[i]) }, 0.0f, 0.0f, 0.0f, 100 + i };
        Body* b = b2o_create_body(e->world, &bd);
        Poly p; b2o_poly_box(&p, (float)hx, (float)hy);
        FixtureDef fd = { &p, 0.0f, 0.2f, 0.0f, 0 };
        b2o_create_fixture(b, &fd);
        e->walls[i] = b;
    }
}

/* RobotPuzzleBase._generate_blocks / _generate_agents / _generate_boundary (core.py:186-243) with
 * Block(shape="T") (blocks.py:68-90) and Robot (robot.py:17-47).  A new Block instance per reset:
 * its vertex list is rebuilt every time (same content). */
static void gen_v3(OrEnv* e, const double* d) {
    const double scale = e->cfg.heavy ? 1.0 : 0.5;            /* core.py:205-210 */
    const double blk_dense = e->cfg.heavy ? V3_DENSE * 2 : V3_DENSE;
    int k = 0;
    {
        BodyDef bd = { BT_DYNAMIC, { (float)d[k], (float)d[k + 1] }, (float)d[k + 2], (float)V3_DAMP, (float)V3_DAMP, 0 };
        k += 3;
        Body* b = b2o_create_body(e->world, &bd);
        add_box_fixture(b, (float)(1 * scale), (float)(1 * scale), 0.0f, (float)(-1 * scale), (float)blk_dense, (float)V3_BLK_FR, 0);
        add_box_fixture(b, (float)(3 * scale), (float)(1 * scale), 0.0f, (float)(1 * scale), (float)blk_dense, (float)V3_BLK_FR, 1);
        e->blocks[0] = b;
        e->nverts[0] = 0; e->verts_init[0] = 0;
        save_vertices(e, 0);
    }
    /* AGENT_POLY robot.py:7-10 scaled by 8 (Python floats, then b2Vec2) */
    static const double AP[8][2] = { { -0.039, -0.095 }, { 0.039, -0.095 }, { 0.095, -0.039 }, { 0.095, 0.039 },
                                     { 0.039, 0.095 }, { -0.039, 0.095 }, { -0.095, 0.039 }, { -0.095, -0.039 } };
    V2 poly[8];
    for (int i = 0; i < 8; ++i) { poly[i].x = (float)(AP[i][0] * V3_AGT_SCALE); poly[i].y = (float)(AP[i][1] * V3_AGT_SCALE); }
    Poly ap; b2o_poly_set(&ap, poly, 8);
    for (int i = 0; i < e->cfg.n_agents; ++i) {
        BodyDef bd = { BT_DYNAMIC, { (float)d[k], (float)d[k + 1] }, 0.0f, 0.0f, 0.0f, 10 + i };   /* no damping (robot.py:42-43) */
        k += 2;
        Body* b = b2o_create_body(e->world, &bd);
        FixtureDef fd = { &ap, (float)V3_AGT_DENSE, 0.2f, 0.0f, 0 };   /* fixtureDef: density 5, friction default 0.2 */
        b2o_create_fixture(b, &fd);
        e->agents[i] = b; e->goal_contact[i] = 0;
    }
    const double bx[4] = { 0, 1, 0.5, 0.5 }, by[4] = { 0.5, 0.5, 0, 1 };
    for (int i = 0; i < 4; ++i) {   /* _generate_boundary core.py:186-201, thickness BORDER */
        double hx = i < 2 ? V3_BORDER : (double)V3_VW / V3_SCALE;
        double hy = i < 2 ? (double)V3_VH / V3_SCALE : V3_BORDER;
        BodyDef bd = { BT_STATIC, { (float)((double)V3_VW / V3_SCALE * bx[i]), (float)((double)V3_VH / V3_SCALE * by[i]) }, 0.0f, 0.0f, 0.0f, 100 + i };
        Body* b = b2o_create_body(e->world, &bd);
        Poly p; b2o_poly_box(&p, (float)hx, (float)hy);
        FixtureDef fd = { &p, 0.0f, 0.2f, 0.0f, 0 };
        b2o_create_fixture(b, &fd);
        e->walls[i] = b;
    }
}

static void gen_v2(OrEnv* e, const double* d) {
    const double vw = (double)V2_VW / V2_SCALE, vh = (double)V2_VH / V2_SCALE;
    double density = e->cfg.heavy ? 20.0 : V2_BLK_DENSE;   /* _02.py:162-165 */
    int k = 0;
    /* _generate_blocks _02.py:313-350 (SIMPLE: fixed position, random angle) */
    for (int i = 0; i < e->cfg.n_blocks; ++i) {
        double x = vw / 2, y = vh / 2;
        if (e->cfg.n_blocks == 3) y += (i == 1 ? 0.4 : (i == 2 ? -0.4 : 0.0));   /* build-defined 3-block layout */
        BodyDef bd = { BT_DYNAMIC, { (float)x, (float)y }, (float)d[k], (float)V2_DAMP, (float)V2_DAMP, i };
        k += 1;
        Body* b = b2o_create_body(e->world, &bd);
        if (i == 0) {
            add_box_fixture(b, 0.1f, 0.1f, 0.0f, -0.1f, (float)density, (float)V2_FR, 0);
            add_box_fixture(b, 0.3f, 0.1f, 0.0f, 0.1f, (float)density, (float)V2_FR, 1);
        } else if (i == 1) {   /* L block: blocks.py:92-102 at scale 0.1 */
            add_box_fixture(b, 0.1f, 0.1f, 0.1f, 0.05f, (float)density, (float)V2_FR, 0);
            add_box_fixture(b, 0.1f, 0.2f, -0.1f, -0.05f, (float)density, (float)V2_FR, 1);
        } else {               /* I block: blocks.py:104-110 at scale 0.1 */
            Poly p; b2o_poly_box(&p, 0.1f, 0.2f);
            FixtureDef fd = { &p, (float)density, (float)V2_FR, 0.0f, 0 };
            b2o_create_fixture(b, &fd);
        }
        e->blocks[i] = b;
        save_vertices(e, i);
    }
    /* _generate_agents _02.py:352-392 */
    V2 poly[8] = { { -0.039f, -0.095f }, { 0.039f, -0.095f }, { 0.095f, -0.039f }, { 0.095f, 0.039f },
                   { 0.039f, 0.095f }, { -0.039f, 0.095f }, { -0.095f, 0.039f }, { -0.095f, -0.039f } };
    Poly ap; b2o_poly_set(&ap, poly, 8);
    Poly w1, w2;
    b2o_poly_box_oriented(&w1, 0.005f, 0.05f, (V2){ 0.06f, 0.0f }, 0.0f);
    b2o_poly_box_oriented(&w2, 0.005f, 0.05f, (V2){ -0.06f, 0.0f }, 0.0f);
    float theta = (float)(3.0 / 2.0 * PY_PI);
    for (int i = 0; i < e->cfg.n_agents; ++i) {
        BodyDef bd = { BT_DYNAMIC, { (float)d[k], (float)d[k + 1] }, theta, (float)V2_DAMP, (float)V2_DAMP, 10 + i };
        k += 2;
        Body* b = b2o_create_body(e->world, &bd);
        FixtureDef f0 = { &ap, (float)V2_AGT_DENSE, (float)V2_FR, 0.0f, 0 };
        FixtureDef f1 = { &w1, 0.0f, (float)V2_FR, 0.0f, 1 };
        FixtureDef f2 = { &w2, 0.0f, (float)V2_FR, 0.0f, 2 };
        b2o_create_fixture(b, &f0); b2o_create_fixture(b, &f1); b2o_create_fixture(b, &f2);
        e->agents[i] = b; e->goal_contact[i] = 0;
    }
    /* _generate_boundary _02.py:394-411 */
    const double bx[4] = { 0, 1, 0.5, 0.5 }, by[4] = { 0.5, 0.5, 0, 1 };
    for (int i = 0; i < 4; ++i) {
        double hx = i < 2 ? V2_BOUNDS : vw;
        double hy = i < 2 ? vh : V2_BOUNDS;
        BodyDef bd = { BT_STATIC, { (float)(vw * bx[i]), (float)(vh * by[i]) }, 0.0f, 0.0f, 0.0f, 100 + i };
        Body* b = b2o_create_body(e->world, &bd);
        Poly p; b2o_poly_box(&p, (float)hx, (float)hy);
        FixtureDef fd = { &p, 0.0f, 0.2f, 0.0f, 0 };
        b2o_create_fixture(b, &fd);
        e->walls[i] = b;
    }
    /* _set_random_goal _02.py:303-311 (draws already mapped to [low, high)) */
    const double ratio = V2_SCALE / V2_VW;
    double gx = d[k], gy = d[k + 1];
    e->goal[0][0] = gx * ratio; e->goal[0][1] = gy * ratio; e->goal[0][2] = 0.0;
    if (e->cfg.n_blocks == 3) {   /* build-defined square: v0 comment offsets (:86-87) x 0.2 m, relative to T */
        double lox = -2.0 / 3.0 * 0.2, loy = (-2.0 / 3.0 - 0.75) * 0.2;
        double iox = 1.0 * 0.2, ioy = (-0.5 - 0.75) * 0.2;
        e->goal[1][0] = (gx + lox) * ratio; e->goal[1][1] = (gy + loy) * ratio; e->goal[1][2] = 0.5 * PY_PI;
        e->goal[2][0] = (gx + iox) * ratio; e->goal[2][1] = (gy + ioy) * ratio; e->goal[2][2] = 0.0;
    }
}

/* _calculate_distance / _calculate_agent_distance: v0 :277-291, v2 _02.py:263-277 */
/* RobotPuzzleBase._get_norm_pose (core.py:289-295): x, y over width_scale, angle mod 2 pi */
static void v3_norm_pose(const Body* b, double* x, double* y) {
    const double ws = (double)V3_VW / V3_SCALE / 2, hs = (double)V3_VH / V3_SCALE / 2;
    *x = ((double)b->sweep.c.x - ws) / ws;
    *y = ((double)b->sweep.c.y - hs) / ws;
}
static void calc_distances(OrEnv* e) {
    if (e->cfg.version == 3) {   /* the distances _get_obs (core.py:297-350) stores */
        double bx, by; v3_norm_pose(e->blocks[0], &bx, &by);
        for (int i = 0; i < e->cfg.n_agents; ++i) {
            double ax, ay; v3_norm_pose(e->agents[i], &ax, &ay);
            e->agent_dist[i] = py_distance(ax, ay, bx, by);
        }
        double gx = (e->goal[0][0] - (double)V3_VW / 2) / ((double)V3_VW / 2);
        double gy = (e->goal[0][1] - (double)V3_VH / 2) / ((double)V3_VW / 2);
        e->block_distance[0] = py_distance(bx, by, gx, gy);
        return;
    }
    if (e->cfg.version == 0) {
        for (int bi = 0; bi < e->cfg.n_blocks; ++bi) {
            V2 c = e->blocks[bi]->sweep.c;
            float sx = c.x * (float)V0_SCALE, sy = c.y * (float)V0_SCALE;   /* b2Vec2 * SCALE in float32 */
            e->block_distance[bi] = py_distance(sx, sy, e->goal[bi][0], e->goal[bi][1]);
        }
        V2 bc = e->blocks[0]->sweep.c;
        float bsx = bc.x * (float)V0_SCALE, bsy = bc.y * (float)V0_SCALE;
        for (int i = 0; i < e->cfg.n_agents; ++i) {
            V2 c = e->agents[i]->sweep.c;
            float ax = c.x * (float)V0_SCALE, ay = c.y * (float)V0_SCALE;
            e->agent_dist[i] = py_distance(ax, ay, bsx, bsy);
        }
    } else {
        const double ratio = V2_SCALE / V2_VW;
        for (int bi = 0; bi < e->cfg.n_blocks; ++bi) {
            V2 c = e->blocks[bi]->sweep.c;
            e->block_distance[bi] = py_distance((double)c.x * ratio, (double)c.y * ratio, e->goal[bi][0], e->goal[bi][1]);
        }
        V2 bc = e->blocks[0]->sweep.c;
        for (int i = 0; i < e->cfg.n_agents; ++i) {
            V2 c = e->agents[i]->sweep.c;
            e->agent_dist[i] = py_distance((double)c.x * ratio, (double)c.y * ratio, (double)bc.x * ratio, (double)bc.y * ratio);
        }
    }
}

/* unitVector :134-138 (Python floats, L-inf normalisation) */
static void unit_vector(const Body* a, const Body* b, double* ux, double* uy) {
    double Ax = a->sweep.c.x, Ay = a->sweep.c.y, Bx = b->sweep.c.x, By = b->sweep.c.y;
    double dx = fabs(Bx - Ax), dy = fabs(By - Ay);
    double denom = dy > dx ? dy : dx;
    *ux = (Bx - Ax) / denom; *uy = (By - Ay) / denom;
}

static void apply_actions(OrEnv* e, const float* action) {
    Body* goal = e->blocks[0];
    if (e->cfg.version == 3) {   /* core.py:353-364, Robot.step robot.py:65-68 */
        for (int i = 0; i < e->cfg.n_agents; ++i) {
            Body* ag = e->agents[i];
            float x = action[3 * i], y = action[3 * i + 1], turn = action[3 * i + 2];
            b2o_set_linear_velocity(ag, (V2){ (float)((double)x * V3_MAX_SPEED), (float)((double)y * V3_MAX_SPEED) });
            b2o_set_angular_velocity(ag, (float)(double)turn);
            double force = py_pow(1.1, -e->agent_dist[i]);
            double ux, uy; unit_vector(ag, goal, &ux, &uy);
            b2o_apply_force(goal, (V2){ (float)(force * ux), (float)(force * uy) }, goal->sweep.c);   /* Block.apply_soft_force */
        }
        return;
    }
    if (e->cfg.version == 0) {
        const double SPEED = 10.0 / V0_SCALE * 4;   /* :50 */
        for (int i = 0; i < e->cfg.n_agents; ++i) {   /* :415-424 */
            Body* ag = e->agents[i];
            float x = action[3 * i], y = action[3 * i + 1], turn = action[3 * i + 2];
            b2o_set_linear_velocity(ag, (V2){ (float)((double)x * SPEED), (float)((double)y * SPEED) });
            b2o_set_angular_velocity(ag, (float)(double)turn);
            double force = py_pow(1.1, -e->agent_dist[i]);
            double ux, uy; unit_vector(ag, goal, &ux, &uy);
            b2o_apply_force(goal, (V2){ (float)(force * ux), (float)(force * uy) }, goal->sweep.c);
        }
    } else {
        for (int i = 0; i < e->cfg.n_agents; ++i) {   /* _02.py:446-474 */
            Body* ag = e->agents[i];
            float turn = action[2 * i], vel = action[2 * i + 1];
            V2 f = b2o_world_vector(ag, (V2){ 0.0f, 1.0f });
            V2 p = b2o_world_point(ag, (V2){ 0.0f, 2.0f });
            double fx = (double)f.x * (double)vel * V2_FORCE, fy = (double)f.y * (double)vel * V2_FORCE;
            b2o_apply_force(ag, (V2){ (float)fx, (float)fy }, p);
            /* updateFriction :116-122 -- pybox2d b2Vec2 ops are float32 */
            V2 n = b2o_world_vector(ag, (V2){ 1.0f, 0.0f });
            float dlat = n.x * ag->v.x + n.y * ag->v.y;
            V2 lat = { n.x * dlat, n.y * dlat };
            V2 nl = { -lat.x, -lat.y };
            V2 imp = { nl.x * ag->mass, nl.y * ag->mass };
            b2o_apply_linear_impulse(ag, imp, ag->sweep.c);
            b2o_apply_angular_impulse(ag, (float)(0.1 * (double)b2o_inertia(ag) * (double)ag->w));
            double torque = (double)fabsf(turn) * 0.0005;
            double tsel = turn;
            if (fabs((double)vel) < 0.1) tsel = 0.0;
            if (tsel < 0) b2o_apply_torque(ag, (float)torque);
            else if (tsel > 0) b2o_apply_torque(ag, (float)(-torque));
            else b2o_apply_torque(ag, 0.0f);
            double force = py_pow(10.0, -e->agent_dist[i]);
            force /= 50;
            double ux, uy; unit_vector(ag, goal, &ux, &uy);
            b2o_apply_force(goal, (V2){ (float)(force * ux), (float)(force * uy) }, goal->sweep.c);
        }
    }
}

static const double TWO_PI = 6.283185307179586;   /* 2*np.pi */

static void build_obs_and_reward(OrEnv* e, const double* prev_agent, const double* prev_block, double* obs, double* reward_out, int* done_out, int* kind_out) {
    int k = 0;
    const Cfg* cfg = &e->cfg;
    Body* goal = e->blocks[0];
    int in_place[3];
    double reward = 0.0; int done = 0, kind = 0;
    if (cfg->version == 3) {
        /* _get_obs core.py:297-350 */
        const double ws = (double)V3_VW / V3_SCALE / 2, hs = (double)V3_VH / V3_SCALE / 2;
        double bx, by; v3_norm_pose(goal, &bx, &by);
        double brot = py_mod((double)goal->sweep.a, TWO_PI);
        for (int i = 0; i < cfg->n_agents; ++i) {
            double ax, ay; v3_norm_pose(e->agents[i], &ax, &ay);
            double arot = py_mod((double)e->agents[i]->sweep.a, TWO_PI);
            obs[k++] = bx - ax; obs[k++] = by - ay; obs[k++] = arot;
            obs[k++] = e->goal_contact[i] ? 1.0 : 0.0;
        }
        double gx = (e->goal[0][0] - (double)V3_VW / 2) / ((double)V3_VW / 2);
        double gy = (e->goal[0][1] - (double)V3_VH / 2) / ((double)V3_VW / 2);
        double grot = py_mod(e->goal[0][2], TWO_PI);
        obs[k++] = gx - bx; obs[k++] = gy - by; obs[k++] = grot - brot;
        for (int j = 0; j < e->nverts[0]; ++j) {   /* Block.get_vertices with norm_fn */
            V2 wp = b2o_world_point(goal, e->verts[0][j]);
            obs[k++] = ((double)wp.x - ws) / ws; obs[k++] = ((double)wp.y - hs) / ws;
        }
        /* step core.py:369-414 */
        int in_place0 = e->block_distance[0] <= V3_EPSILON / (double)V3_VW * 2;
        double deltaDist = prev_block[0] - e->block_distance[0];
        reward += deltaDist * e->w_dBlock;
        reward -= e->w_blkDist * e->block_distance[0];
        for (int i = 0; i < cfg->n_agents; ++i) {
            double deltaAgent = prev_agent[i] - e->agent_dist[i];
            reward += deltaAgent * e->w_dAgent / 4.;
            reward -= e->w_agentDist * e->agent_dist[i] / 4.;
            if (e->goal_contact[i]) reward += 0.25;
        }
        if (in_place0) { done = 1; kind = 1; reward += e->puzzle_complete; }
    } else if (cfg->version == 0) {
        /* obs :442-472 */
        for (int i = 0; i < cfg->n_agents; ++i) {
            double x = goal->sweep.c.x, y = goal->sweep.c.y;
            V2 ac = e->agents[i]->sweep.c;
            obs[k++] = (double)ac.x * V0_SCALE - x * V0_SCALE;
            obs[k++] = (double)ac.y * V0_SCALE - y * V0_SCALE;
            obs[k++] = e->agent_dist[i];
            obs[k++] = e->goal_contact[i] ? 1.0 : 0.0;
        }
        for (int bi = 0; bi < cfg->n_blocks; ++bi) {
            Body* b = e->blocks[bi];
            double x = b->sweep.c.x, y = b->sweep.c.y;
            double angle = py_mod((double)b->sweep.a, TWO_PI);
            double fx = e->goal[bi][0], fy = e->goal[bi][1], fangle = e->goal[bi][2];
            x *= V0_SCALE; y *= V0_SCALE;
            double a_diff = py_mod(fangle, TWO_PI) - angle;
            in_place[bi] = !(fabs(fx - x) > V0_EPSILON) && !(fabs(fy - y) > V0_EPSILON);   /* is_in_place :380-386 */
            obs[k++] = x - fx; obs[k++] = y - fy; obs[k++] = a_diff;
            obs[k++] = py_distance(x, y, fx, fy);
            for (int j = 0; j < e->nverts[bi]; ++j) {
                V2 wp = b2o_world_point(b, e->verts[bi][j]);
                obs[k++] = (double)wp.x * V0_SCALE; obs[k++] = (double)wp.y * V0_SCALE;
            }
        }
        /* reward :475-519 */
        double deltaDist = prev_block[0] - e->block_distance[0];
        reward += deltaDist * e->w_dBlock * 1.0 / 4.;
        reward -= e->w_blkDist * e->block_distance[0] * 1.0 / 4.;
        for (int i = 0; i < cfg->n_agents; ++i) {
            double deltaAgent = prev_agent[i] - e->agent_dist[i];
            reward += deltaAgent * e->w_dAgent * 1.0 / 4.;
            reward -= e->w_agentDist * e->agent_dist[i] * 1.0 / 4.;
            if (e->goal_contact[i]) reward += 0.25;
        }
        e->prev_blks_in_place = e->blks_in_place;
        e->blks_in_place = 0;
        for (int bi = 0; bi < cfg->n_blocks; ++bi) if (in_place[bi]) e->blks_in_place += 1;
        reward += (double)((e->blks_in_place - e->prev_blks_in_place) * 10);
        if (e->blks_in_place == 1) { done = 1; kind = 1; reward += 10000; }
    } else {
        const double ratio = V2_SCALE / V2_VW;
        /* obs _02.py:494-532 */
        for (int i = 0; i < cfg->n_agents; ++i) {
            Body* ag = e->agents[i];
            double aX = (double)ag->sweep.c.x * ratio, aY = (double)ag->sweep.c.y * ratio;
            double theta = py_mod((double)ag->sweep.a, TWO_PI);
            double nt = theta <= PY_PI ? -theta / PY_PI : (TWO_PI - theta) / PY_PI;   /* norm_angle :255-261 */
            double bX = (double)goal->sweep.c.x * ratio, bY = (double)goal->sweep.c.y * ratio;
            obs[k++] = aX; obs[k++] = aY; obs[k++] = nt;
            obs[k++] = aX - bX; obs[k++] = aY - bY;
            obs[k++] = ag->v.x; obs[k++] = ag->v.y; obs[k++] = ag->w;
            obs[k++] = e->agent_dist[i];
        }
        for (int bi = 0; bi < cfg->n_blocks; ++bi) {
            Body* b = e->blocks[bi];
            double x = (double)b->sweep.c.x * ratio, y = (double)b->sweep.c.y * ratio;
            double angle = py_mod((double)b->sweep.a, TWO_PI);
            double fx = e->goal[bi][0], fy = e->goal[bi][1], fangle = e->goal[bi][2];
            double a_diff = py_mod(fangle, TWO_PI) - angle;
            a_diff /= PY_PI;
            in_place[bi] = !(fabs(fx - x) > e->scaled_epsilon) && !(fabs(fy - y) > e->scaled_epsilon);
            obs[k++] = x - fx; obs[k++] = y - fy; obs[k++] = a_diff;
            obs[k++] = py_distance(x, y, fx, fy);
            for (int j = 0; j < e->nverts[bi]; ++j) {
                V2 wp = b2o_world_point(b, e->verts[bi][j]);
                obs[k++] = (double)wp.x * ratio; obs[k++] = (double)wp.y * ratio;
            }
        }
        obs[k++] = e->scaled_epsilon;   /* contact_weight :531-532 */
        /* reward _02.py:535-584 */
        double deltaDist = prev_block[0] - e->block_distance[0];
        reward += deltaDist * e->w_dBlock;
        reward -= e->w_blkDist * e->block_distance[0];
        for (int i = 0; i < cfg->n_agents; ++i) {
            double deltaAgent = prev_agent[i] - e->agent_dist[i];
            reward += deltaAgent * e->w_dAgent;
            reward -= e->w_agentDist * e->agent_dist[i];
        }
        const double vw = (double)V2_VW / V2_SCALE, vh = (double)V2_VH / V2_SCALE;
        int agt_oob = 0, blk_oob = 0;
        for (int i = 0; i < cfg->n_agents && !agt_oob; ++i) {   /* _agt_out_of_bounds :288-295 */
            double x = e->agents[i]->sweep.c.x, y = e->agents[i]->sweep.c.y;
            if (x < V2_BOUNDS || x > (vw - V2_BOUNDS)) agt_oob = 1;
            else if (y < V2_BOUNDS || y > (vh - V2_BOUNDS)) agt_oob = 1;
        }
        for (int bi = 0; bi < cfg->n_blocks && !blk_oob; ++bi) {   /* _blk_out_of_bounds :279-286 */
            double x = e->blocks[bi]->sweep.c.x, y = e->blocks[bi]->sweep.c.y;
            if (x < V2_BOUNDS || x > (vw - V2_BOUNDS)) blk_oob = 1;
            else if (y < V2_BOUNDS || y > (vh - V2_BOUNDS)) blk_oob = 1;
        }
        if (agt_oob) { done = 1; kind = 2; reward -= e->shaped_bounds; }
        else if (blk_oob) { done = 1; kind = 3; reward -= e->shaped_blk_bounds; }
        else {
            e->prev_blks_in_place = e->blks_in_place;
            e->blks_in_place = 0;
            for (int bi = 0; bi < cfg->n_blocks; ++bi) if (in_place[bi]) e->blks_in_place += 1;
            int num_in_contact = 0;
            for (int i = 0; i < cfg->n_agents; ++i) if (e->goal_contact[i]) num_in_contact += 1;
            if (e->blks_in_place == cfg->n_blocks) {
                done = 1; kind = 1;
                reward += e->shaped_puzzle * ((double)num_in_contact / (double)cfg->n_agents);
            }
        }
    }
    *reward_out = reward; *done_out = done; *kind_out = kind;
}

void or_step(OrEnv* e, const float* action, double* obs, double* reward, int* done, int* kind) {
    apply_actions(e, action);
    /* for _ in range(self.frameskip): world.Step(1.0/FPS, 6*30, 2*30)  (_02.py:476-478; v0 :427-428 with
     * frameskip 1 for the low-dim obs, :161-162); forces are cleared after the first Step */
    for (int f = 0; f < (e->frameskip > 0 ? e->frameskip : 1); ++f) b2o_step(e->world, 1.0f / 50, 6 * 30, 2 * 30);
    double prev_agent[5], prev_block[3];
    memcpy(prev_agent, e->agent_dist, sizeof(prev_agent));
    memcpy(prev_block, e->block_distance, sizeof(prev_block));
    calc_distances(e);
    build_obs_and_reward(e, prev_agent, prev_block, obs, reward, done, kind);
}

/* reset multi_robot_puzzle_00.py:392-411 / _02.py:421-442 */
void or_reset(OrEnv* e, const double* draws, const float* reset_action, double* obs_out) {
    env_destroy_bodies(e);
    b2o_set_listener(e->world, cb_begin, cb_end, e);
    if (e->cfg.version == 0) gen_v0(e, draws); else if (e->cfg.version == 3) gen_v3(e, draws); else gen_v2(e, draws);
    e->have_bodies = 1;
    calc_distances(e);
    double reward; int done, kind;
    or_step(e, reset_action, obs_out, &reward, &done, &kind);
}

int or_get_bodies(const OrEnv* e, float* out) {
    int k = 0;
    for (int i = 0; i < e->cfg.n_blocks; ++i) {
        const Body* b = e->blocks[i];
        out[k++] = b->sweep.c.x; out[k++] = b->sweep.c.y; out[k++] = b->sweep.a;
        out[k++] = b->v.x; out[k++] = b->v.y; out[k++] = b->w;
    }
    for (int i = 0; i < e->cfg.n_agents; ++i) {
        const Body* b = e->agents[i];
        out[k++] = b->sweep.c.x; out[k++] = b->sweep.c.y; out[k++] = b->sweep.a;
        out[k++] = b->v.x; out[k++] = b->v.y; out[k++] = b->w;
    }
    return k;
}
void or_get_flags(const OrEnv* e, int* gc, int* bip) {
    for (int i = 0; i < e->cfg.n_agents; ++i) gc[i] = e->goal_contact[i];
    *bip = e->blks_in_place;
}
int or_contact_count(const OrEnv* e) { return e->world->cm.contactCount; }
void or_set_frameskip(OrEnv* e, int frameskip) { e->frameskip = frameskip; }
void or_counters(const OrEnv* e, long* toi, long* pos) { *toi = e->world->toiEvents; *pos = e->world->posIters; }
void or_capacity(const OrEnv* e, int* out8) {
    const World* w = e->world;
    out8[0] = w->cm.maxContacts; out8[1] = w->cm.bp.tree.maxId; out8[2] = w->cm.bp.maxMove;
    out8[3] = w->maxIslandBodies; out8[4] = w->maxIslandContacts; out8[5] = w->maxToiIslandBodies;
    out8[6] = w->maxToiIslandContacts; out8[7] = w->cm.bp.tree.nodeCapacity;
}
void or_work(const OrEnv* e, long* out20) {
    OrWork k = e->world->work;
    k.sat_calls = e->world->cm.satCalls;
    const long* v = (const long*)&k;
    for (int i = 0; i < 20; ++i) out20[i] = v[i];
}
void or_counters_ex(const OrEnv* e, long* out3) {
    out3[0] = e->world->toiEvents; out3[1] = e->world->posIters; out3[2] = e->world->touching;
}
long or_vel_constraint_iters(const OrEnv* e) { return e->world->velIters; }
static int push_proxies(const Body* b, int* out, int k) {
    /* creation order == reverse fixture-list order */
    int n = 0; const Fixture* fs[8];
    for (const Fixture* f = b->fixtureList; f; f = f->next) fs[n++] = f;
    for (int i = n - 1; i >= 0; --i) out[k++] = fs[i]->proxyId;
    return k;
}
int or_proxy_ids(const OrEnv* e, int* out) {
    int k = 0;
    for (int i = 0; i < e->cfg.n_blocks; ++i) k = push_proxies(e->blocks[i], out, k);
    for (int i = 0; i < e->cfg.n_agents; ++i) k = push_proxies(e->agents[i], out, k);
    for (int i = 0; i < 4; ++i) k = push_proxies(e->walls[i], out, k);
    return k;
}

/* Mass data of dynamic body i (blocks, then agents): mass, rotational inertia about the
 * body origin (b2Body::GetInertia), local centre x, y.  Known-answer tests. */
int or_body_mass(const OrEnv* e, int i, float* out4) {
    int nb = e->cfg.n_blocks, na = e->cfg.n_agents;
    if (!e->have_bodies || i < 0 || i >= nb + na) return -1;
    const Body* b = i < nb ? e->blocks[i] : e->agents[i - nb];
    out4[0] = b->mass; out4[1] = b2o_inertia(b);
    out4[2] = b->sweep.localCenter.x; out4[3] = b->sweep.localCenter.y;
    return 0;
}

/* Batched run with the device path's synthetic-input scheme (mrp_kernels.hip k_step/k_reset,
 * actions == NULL, draws == NULL, auto-reset on): lane l is global lane lane_offset + l;
 * reset e of a lane draws spawn d from RNG stream 1 and its action component j from stream 2
 * (counter e*64 + d / j); step s of a lane (counted over the lane's lifetime) takes action
 * component j from stream 3 (counter s*64 + j); done or TimeLimit -> reset.  Lanes are split
 * over `threads` OpenMP threads.  Used as bench.py's CPU baseline and as the full-size parity
 * checker of the device auto-reset path.  Returns env-steps done; *seconds = wall time of the
 * stepping loop (initial resets and env creation excluded).  Optional outputs (NULL to skip):
 * max_steps <= 0 uses the registered TimeLimit.  bodies [n_lanes][6*(n_blocks+n_agents)] final state, rsum [n_lanes] summed float32(reward),
 * resets [n_lanes] episodes started. */
#include <omp.h>
static long batch_run(int env_id, int n_lanes, int skip, int steps, uint64_t seed, uint64_t lane_offset, const double* lo,
                      const double* hi, int max_steps, int threads, double* seconds, float* bodies, double* rsum,
                      int* resets, int* caps, long* work);
long or_batch_run(int env_id, int n_lanes, int steps, uint64_t seed, uint64_t lane_offset, const double* lo,
                  const double* hi, int max_steps, int threads, double* seconds, float* bodies, double* rsum,
                  int* resets) {
    return batch_run(env_id, n_lanes, 0, steps, seed, lane_offset, lo, hi, max_steps, threads, seconds, bodies, rsum, resets,
                     NULL, NULL);
}
/* or_batch_run with `skip` untimed steps first: *seconds times only steps skip+1 .. skip+steps of
 * every lane (bench.py's CPU baseline on the GPU line's step window); returns the timed env-steps */
long or_batch_run_window(int env_id, int n_lanes, int skip, int steps, uint64_t seed, uint64_t lane_offset, const double* lo,
                         const double* hi, int max_steps, int threads, double* seconds, float* bodies, double* rsum,
                         int* resets) {
    return batch_run(env_id, n_lanes, skip, steps, seed, lane_offset, lo, hi, max_steps, threads, seconds, bodies, rsum, resets,
                     NULL, NULL);
}
long or_batch_capacity(int env_id, int n_lanes, int steps, uint64_t seed, const double* lo, const double* hi, int max_steps,
                       int threads, int* caps8) {
    double sec;
    for (int k = 0; k < 8; ++k) caps8[k] = 0;
    return batch_run(env_id, n_lanes, 0, steps, seed, 0, lo, hi, max_steps, threads, &sec, NULL, NULL, NULL, caps8, NULL);
}
long or_batch_work(int env_id, int n_lanes, int steps, uint64_t seed, const double* lo, const double* hi, int max_steps,
                   int threads, long* work) {
    double sec;
    return batch_run(env_id, n_lanes, 0, steps, seed, 0, lo, hi, max_steps, threads, &sec, NULL, NULL, NULL, NULL, work);
}
/* the build's name for the solver variant it was compiled as (bench.py records it) */
const char* or_build_kind(void) {
#if defined(OR_NO_WORK) && defined(OR_EARLY_EXIT)
    return "early-exit port: work model compiled out, velocity sweeps stop at the device's exact period-1/2 exit";
#elif defined(OR_NO_WORK)
    return "port: work model compiled out, all 180 velocity sweeps (b2Island::Solve)";
#else
    return "checker: work model compiled in";
#endif
}
static long batch_run(int env_id, int n_lanes, int skip, int steps, uint64_t seed, uint64_t lane_offset, const double* lo,
                      const double* hi, int max_steps, int threads, double* seconds, float* bodies, double* rsum,
                      int* resets, int* caps, long* work) {
    if (!valid(env_id) || n_lanes <= 0 || steps < 0 || skip < 0) return -1;
    const Cfg cfg = CFGS[env_id];
    const int limit = max_steps > 0 ? max_steps : cfg.max_steps;
    const int nbody = 6 * (cfg.n_blocks + cfg.n_agents);
    OrEnv** envs = (OrEnv**)calloc((size_t)n_lanes, sizeof(OrEnv*));
    int* episode = (int*)calloc((size_t)n_lanes, sizeof(int));
    int* elapsed = (int*)calloc((size_t)n_lanes, sizeof(int));
    double* rs = (double*)calloc((size_t)n_lanes, sizeof(double));
    if (threads > 0) omp_set_num_threads(threads);
    double t0 = 0.0, t1 = 0.0;
    long total = 0;
#pragma omp parallel
    {
        double draws[16], obs[128], rew; float act[16]; int done, kind;
#pragma omp for schedule(static)
        for (int l = 0; l < n_lanes; ++l) {
            const uint64_t g = lane_offset + (uint64_t)l;
            envs[l] = or_create(env_id);
            for (int d = 0; d < cfg.n_draws; ++d) draws[d] = lo[d] + (hi[d] - lo[d]) * or_rng_u01(seed, g, 1, (uint64_t)d);
            for (int j = 0; j < cfg.act_dim; ++j) act[j] = (float)(-1.0 + 2.0 * or_rng_u01(seed, g, 2, (uint64_t)j));
            or_reset(envs[l], draws, act, obs);
            episode[l] = 1;
        }
        /* phase 0: the untimed steps [0, skip); phase 1: the timed steps [skip, skip + steps) */
        for (int phase = 0; phase < 2; ++phase) {
            const int s0 = phase ? skip : 0, s1 = phase ? skip + steps : skip;
            if (s1 <= s0) continue;
#pragma omp barrier
#pragma omp single
            t0 = omp_get_wtime();
            /* dynamic: a lane's cost varies by orders of magnitude between steps (contact islands), and
             * lanes are independent, so the CPU baseline takes the best balance it can */
#pragma omp for schedule(dynamic, 4) reduction(+:total)
            for (int l = 0; l < n_lanes; ++l) {
                OrEnv* e = envs[l];
                const uint64_t g = lane_offset + (uint64_t)l;
                for (int s = s0; s < s1; ++s) {
                    for (int j = 0; j < cfg.act_dim; ++j)
                        act[j] = (float)(-1.0 + 2.0 * or_rng_u01(seed, g, 3, (uint64_t)s * 64 + (uint64_t)j));
                    long w0[20];
                    if (work) or_work(e, w0);
                    or_step(e, act, obs, &rew, &done, &kind);
                    rs[l] += (double)(float)rew;
                    if (phase) ++total;
                    if (done || ++elapsed[l] >= limit) {
                        const uint64_t ctr = (uint64_t)episode[l] * 64;
                        for (int d = 0; d < cfg.n_draws; ++d)
                            draws[d] = lo[d] + (hi[d] - lo[d]) * or_rng_u01(seed, g, 1, ctr + (uint64_t)d);
                        for (int j = 0; j < cfg.act_dim; ++j)
                            act[j] = (float)(-1.0 + 2.0 * or_rng_u01(seed, g, 2, ctr + (uint64_t)j));
                        or_reset(e, draws, act, obs);
                        ++episode[l];
                        elapsed[l] = 0;
                    }
                    if (work) {   /* this launch's work for the lane: the step plus an auto-reset's own step */
                        long w1[20];
                        or_work(e, w1);
                        for (int k = 0; k < 20; ++k) work[((size_t)s * n_lanes + l) * 20 + k] = w1[k] - w0[k];
                    }
                }
            }
#pragma omp single
            t1 = omp_get_wtime();
        }
#pragma omp for schedule(static)
        for (int l = 0; l < n_lanes; ++l)
            if (rsum) rsum[l] = rs[l];
#pragma omp for schedule(static)
        for (int l = 0; l < n_lanes; ++l) {
            if (bodies) or_get_bodies(envs[l], bodies + (size_t)l * nbody);
            if (resets) resets[l] = episode[l];
            if (caps) {
                int c[8];
                or_capacity(envs[l], c);
#pragma omp critical
                for (int k = 0; k < 8; ++k) if (c[k] > caps[k]) caps[k] = c[k];
            }
            or_destroy(envs[l]);
        }
    }
    *seconds = t1 - t0;
    free(envs); free(episode); free(elapsed); free(rs);
    return total;
}
