// mrp_tables.cpp -- host-side construction of the per-env static tables: polygon hulls
// and normals (b2PolygonShape::Set / SetAsBox), mass data (ComputeMass + ResetMassData),
// fixture/body layout, obs vertex lists and spawn bounds.  float32 arithmetic in Box2D
// v2.3 order (this TU is built with -ffp-contract=off like the kernels).
//
// Geometry sources: multi_robot_puzzle_00.py:62-67,260-275,299-378 (v0),
// multi_robot_puzzle_02.py:64-67,313-411 (v2), blocks.py:80-110 (L/I shapes of the
// build-defined 3-block config), core.py:186-243 + robot.py:7-44 + blocks.py:70-90 (v3).
#include "mrp_tables.h"

#include <cmath>
#include <cstring>

namespace mrp {

static constexpr float POLY_RADIUS = 2.0f * 0.005f;

static void poly_box(ShapeDef& p, float hx, float hy) {
    p.count = 4;
    p.v[0] = v2(-hx, -hy); p.v[1] = v2(hx, -hy); p.v[2] = v2(hx, hy); p.v[3] = v2(-hx, hy);
    p.n[0] = v2(0.0f, -1.0f); p.n[1] = v2(1.0f, 0.0f); p.n[2] = v2(0.0f, 1.0f); p.n[3] = v2(-1.0f, 0.0f);
    p.radius = POLY_RADIUS;
}

static void poly_box_oriented(ShapeDef& p, float hx, float hy, V2 center, float angle) {
    poly_box(p, hx, hy);
    Xf xf; xf.p = center; xf.q = rot(angle);
    for (int i = 0; i < 4; ++i) { p.v[i] = mul_xv(xf, p.v[i]); p.n[i] = mul_rv(xf.q, p.n[i]); }
}

// b2PolygonShape::Set: weld, gift-wrap hull (start at max x, then min y), normals
static void poly_set(ShapeDef& p, const V2* vin, int count) {
    p.radius = POLY_RADIUS;
    V2 ps[MAX_POLY];
    int n = 0;
    for (int i = 0; i < count && i < MAX_POLY; ++i) {
        bool unique = true;
        for (int j = 0; j < n; ++j) {
            V2 d = vsub(vin[i], ps[j]);
            if (vlensq(d) < ((0.5f * 0.005f) * (0.5f * 0.005f))) { unique = false; break; }
        }
        if (unique) ps[n++] = vin[i];
    }
    int i0 = 0; float x0 = ps[0].x;
    for (int i = 1; i < n; ++i) {
        float x = ps[i].x;
        if (x > x0 || (x == x0 && ps[i].y < ps[i0].y)) { i0 = i; x0 = x; }
    }
    int hull[MAX_POLY]; int m = 0; int ih = i0;
    for (;;) {
        hull[m] = ih;
        int ie = 0;
        for (int j = 1; j < n; ++j) {
            if (ie == ih) { ie = j; continue; }
            V2 r = vsub(ps[ie], ps[hull[m]]), v = vsub(ps[j], ps[hull[m]]);
            float c = vcross(r, v);
            if (c < 0.0f) ie = j;
            if (c == 0.0f && vlensq(v) > vlensq(r)) ie = j;
        }
        ++m; ih = ie;
        if (ie == i0) break;
    }
    p.count = m;
    for (int i = 0; i < m; ++i) p.v[i] = ps[hull[i]];
    for (int i = 0; i < m; ++i) {
        V2 edge = vsub(p.v[i + 1 < m ? i + 1 : 0], p.v[i]);
        p.n[i] = vcross_vs(edge, 1.0f);
        vnormalize(p.n[i]);
    }
}

// b2PolygonShape::ComputeMass
static void poly_mass(const ShapeDef& p, float density, float& mass, V2& center_out, float& I_out) {
    V2 center = v2(0.0f, 0.0f);
    float area = 0.0f, I = 0.0f;
    V2 s = v2(0.0f, 0.0f);
    for (int i = 0; i < p.count; ++i) s = vadd(s, p.v[i]);
    { float inv = 1.0f / p.count; s.x *= inv; s.y *= inv; }
    const float k_inv3 = 1.0f / 3.0f;
    for (int i = 0; i < p.count; ++i) {
        V2 e1 = vsub(p.v[i], s);
        V2 e2 = i + 1 < p.count ? vsub(p.v[i + 1], s) : vsub(p.v[0], s);
        float D = vcross(e1, e2);
        float triangleArea = 0.5f * D;
        area += triangleArea;
        center = vadd(center, vmul(triangleArea * k_inv3, vadd(e1, e2)));
        float ex1 = e1.x, ey1 = e1.y, ex2 = e2.x, ey2 = e2.y;
        float intx2 = ex1 * ex1 + ex2 * ex1 + ex2 * ex2;
        float inty2 = ey1 * ey1 + ey2 * ey1 + ey2 * ey2;
        I += (0.25f * k_inv3 * D) * (intx2 + inty2);
    }
    mass = density * area;
    { float inv = 1.0f / area; center.x *= inv; center.y *= inv; }
    center_out = vadd(center, s);
    I_out = density * I;
    I_out += mass * (vdot(center_out, center_out) - vdot(center, center));
}

struct FixSpec { ShapeDef shape; float density, friction; };

// b2Body::ResetMassData over the fixture list (newest fixture first)
static void reset_mass(EnvTables& t, int b, const FixSpec* fx, int nfx) {
    float mass = 0.0f, I = 0.0f;
    V2 lc = v2(0.0f, 0.0f);
    bool any = false;
    for (int k = nfx - 1; k >= 0; --k) {
        if (fx[k].density == 0.0f) continue;
        any = true;
        float m; V2 c; float Ii;
        poly_mass(fx[k].shape, fx[k].density, m, c, Ii);
        mass += m; lc = vadd(lc, vmul(m, c)); I += Ii;
    }
    float invMass = 0.0f, invI = 0.0f;
    if (!any) {   // constructor values of a dynamic body: mass 1, I 0
        t.mass[b] = 1.0f; t.invMass[b] = 1.0f; t.I[b] = 0.0f; t.invI[b] = 0.0f; t.lcx[b] = 0.0f; t.lcy[b] = 0.0f;
        t.body_reset_mass[b] = 0;
        return;
    }
    if (mass > 0.0f) { invMass = 1.0f / mass; lc.x *= invMass; lc.y *= invMass; }
    else { mass = 1.0f; invMass = 1.0f; }
    if (I > 0.0f) { I -= mass * vdot(lc, lc); invI = 1.0f / I; }
    else { I = 0.0f; invI = 0.0f; }
    t.mass[b] = mass; t.invMass[b] = invMass; t.I[b] = I; t.invI[b] = invI; t.lcx[b] = lc.x; t.lcy[b] = lc.y;
    t.body_reset_mass[b] = 1;
}

static void add_body(EnvTables& t, int b, int& nfix, const FixSpec* fx, int n, bool dynamic, float damp) {
    t.body_fix0[b] = nfix; t.body_nfix[b] = n;
    for (int k = 0; k < n; ++k) {
        int f = nfix++;
        t.fix_body[f] = b; t.fix_friction[f] = fx[k].friction; t.fix_restitution[f] = 0.0f; t.shape[f] = fx[k].shape;
    }
    t.linDamp[b] = damp; t.angDamp[b] = damp;
    if (dynamic) reset_mass(t, b, fx, n);
    else { t.mass[b] = 0.0f; t.invMass[b] = 0.0f; t.I[b] = 0.0f; t.invI[b] = 0.0f; t.lcx[b] = 0.0f; t.lcy[b] = 0.0f; t.body_reset_mass[b] = 0; }
}

// "SAVE vertices data": fixture-list order (newest first), duplicates of earlier fixtures skipped
static void save_vertices(EnvTables& t, int bi, const FixSpec* fx, int n) {
    int nv = 0;
    for (int k = n - 1; k >= 0; --k) {
        const ShapeDef& s = fx[k].shape;
        if (k == n - 1) { for (int i = 0; i < s.count; ++i) t.verts[bi][nv++] = s.v[i]; continue; }
        int n0 = nv;
        for (int i = 0; i < s.count; ++i) {
            bool found = false;
            for (int j = 0; j < n0; ++j) if (t.verts[bi][j].x == s.v[i].x && t.verts[bi][j].y == s.v[i].y) { found = true; break; }
            if (!found) t.verts[bi][nv++] = s.v[i];
        }
    }
    t.nverts[bi] = nv;
}

static FixSpec box_fix(float hx, float hy, float cx, float cy, float density, float friction) {
    FixSpec f; std::memset(&f, 0, sizeof(f));
    poly_box_oriented(f.shape, hx, hy, v2(cx, cy), 0.0f);
    f.density = density; f.friction = friction;
    return f;
}

bool build_tables(int env_id, EnvTables& t) {
    if (env_id < 0 || env_id >= N_ENVS) return false;
    std::memset(&t, 0, sizeof(t));
    const EnvCfg& cfg = ENV_CFG[env_id];
    const int na = cfg.n_agents, nb = cfg.n_blocks;
    t.env_id = env_id; t.version = cfg.version;
    t.n_agents = na; t.n_blocks = nb;
    t.n_dyn = t.n_agents + t.n_blocks; t.n_bodies = t.n_dyn + 4;
    // action / spawn-draw layouts: multi_robot_puzzle_00.py:206,311-315,366-367 (3 action values per
    // agent; block x, y, angle + agent x, y), _02.py:194,307-308,324,358-359 (2 per agent; block
    // angles + agent x, y + goal x, y), core.py:136,212-215,231-232 (v3 as v0); obs_dim at the end
    if (cfg.version == 2) { t.act_dim = 2 * na; t.n_draws = nb + 2 * na + 2; }
    else { t.act_dim = 3 * na; t.n_draws = 3 + 2 * na; }
    t.max_steps = cfg.max_steps;
    int nfix = 0;
    const double PI = 3.141592653589793;
    if (t.version == 0) {
        const bool heavy = cfg.heavy != 0;
        const double S = 2.0, scaled = heavy ? S / 2 : S, dense = heavy ? 5.0 * 2 : 5.0;
        FixSpec blk[2] = {box_fix((float)(1 / scaled), (float)(1 / scaled), 0.0f, (float)(-1 / scaled), (float)dense, (float)0.999),
                          box_fix((float)(3 / scaled), (float)(1 / scaled), 0.0f, (float)(1 / scaled), (float)dense, (float)0.999)};
        add_body(t, 0, nfix, blk, 2, true, 5.0f);
        save_vertices(t, 0, blk, 2);
        V2 poly[8] = {{(float)(-0.5 / S), (float)(-1.5 / S)}, {(float)(0.5 / S), (float)(-1.5 / S)}, {(float)(1.5 / S), (float)(-0.5 / S)},
                      {(float)(1.5 / S), (float)(0.5 / S)}, {(float)(0.5 / S), (float)(1.5 / S)}, {(float)(-0.5 / S), (float)(1.5 / S)},
                      {(float)(-1.5 / S), (float)(0.5 / S)}, {(float)(-1.5 / S), (float)(-0.5 / S)}};
        FixSpec ag; std::memset(&ag, 0, sizeof(ag));
        poly_set(ag.shape, poly, 8); ag.density = 0.0f; ag.friction = 0.2f;
        for (int i = 0; i < t.n_agents; ++i) add_body(t, 1 + i, nfix, &ag, 1, true, 5.0f);
        const double vw = 640 / 30.0, vh = 480 / 30.0;
        const double bx[4] = {0, 1, 0.5, 0.5}, by[4] = {0.5, 0.5, 0, 1};
        for (int w = 0; w < 4; ++w) {
            FixSpec wf; std::memset(&wf, 0, sizeof(wf));
            poly_box(wf.shape, (float)(w < 2 ? 1.0 : vw), (float)(w < 2 ? vh : 1.0)); wf.density = 0.0f; wf.friction = 0.2f;
            int b = t.n_dyn + w;
            add_body(t, b, nfix, &wf, 1, false, 0.0f);
            t.wall_px[w] = (float)(vw * bx[w]); t.wall_py[w] = (float)(vh * by[w]);
        }
        t.goal_x = (double)(640 / 2) + 0.0 * 30.0; t.goal_y = (double)(480 / 2) + 0.75 * 30.0; t.goal_a = 0.0;
        const double xr[2] = {1.0, 640 / 30.0 - 1}, yr[2] = {1.0, 480 / 30.0 - 1};
        int k = 0;
        t.draw_lo[k] = xr[0]; t.draw_hi[k++] = xr[1]; t.draw_lo[k] = yr[0]; t.draw_hi[k++] = yr[1];
        t.draw_lo[k] = 0.0; t.draw_hi[k++] = 2 * PI;
        for (int i = 0; i < t.n_agents; ++i) { t.draw_lo[k] = xr[0]; t.draw_hi[k++] = xr[1]; t.draw_lo[k] = yr[0]; t.draw_hi[k++] = yr[1]; }
        t.agent_angle = 0.0f;
    } else if (t.version == 3) {
        // RobotPuzzleBase: Block("T") at scale 0.5 (heavy: 1) density 5 (heavy: 10), friction 2.5,
        // damping 5 (blocks.py:70-90, core.py:204-225); Robot AGENT_POLY * 8, density 5,
        // friction 0.2, no damping (robot.py:34-44); walls as v0 (core.py:186-201)
        const bool heavy = cfg.heavy != 0;
        const double sc = heavy ? 1.0 : 0.5, dense = heavy ? 5.0 * 2 : 5.0;
        FixSpec blk[2] = {box_fix((float)(1 * sc), (float)(1 * sc), 0.0f, (float)(-1 * sc), (float)dense, 2.5f),
                          box_fix((float)(3 * sc), (float)(1 * sc), 0.0f, (float)(1 * sc), (float)dense, 2.5f)};
        add_body(t, 0, nfix, blk, 2, true, 5.0f);
        save_vertices(t, 0, blk, 2);
        static const double AP[8][2] = {{-0.039, -0.095}, {0.039, -0.095}, {0.095, -0.039}, {0.095, 0.039},
                                        {0.039, 0.095}, {-0.039, 0.095}, {-0.095, 0.039}, {-0.095, -0.039}};
        V2 poly[8];
        for (int i = 0; i < 8; ++i) poly[i] = v2((float)(AP[i][0] * 8.0), (float)(AP[i][1] * 8.0));
        FixSpec ag; std::memset(&ag, 0, sizeof(ag));
        poly_set(ag.shape, poly, 8); ag.density = 5.0f; ag.friction = 0.2f;
        for (int i = 0; i < t.n_agents; ++i) add_body(t, 1 + i, nfix, &ag, 1, true, 0.0f);
        const double vw = 640 / 30.0, vh = 480 / 30.0;
        const double bx[4] = {0, 1, 0.5, 0.5}, by[4] = {0.5, 0.5, 0, 1};
        for (int w = 0; w < 4; ++w) {
            FixSpec wf; std::memset(&wf, 0, sizeof(wf));
            poly_box(wf.shape, (float)(w < 2 ? 1.0 : vw), (float)(w < 2 ? vh : 1.0)); wf.density = 0.0f; wf.friction = 0.2f;
            int b = t.n_dyn + w;
            add_body(t, b, nfix, &wf, 1, false, 0.0f);
            t.wall_px[w] = (float)(vw * bx[w]); t.wall_py[w] = (float)(vh * by[w]);
        }
        t.goal_x = 5.0 / 6.0 * 640 - 4.0 / 3.0 * 1; t.goal_y = (double)(480 / 2); t.goal_a = 0.0;   // core.py:277-281
        int k = 0;   // core.py:212-215, 231-232
        t.draw_lo[k] = vw / 3 + 2 * 1; t.draw_hi[k++] = vw * 2 / 3 - 2 * 1;
        t.draw_lo[k] = 3 * 1; t.draw_hi[k++] = vh - 3 * 1;
        t.draw_lo[k] = 0.0; t.draw_hi[k++] = 2 * PI;
        for (int i = 0; i < t.n_agents; ++i) { t.draw_lo[k] = 1; t.draw_hi[k++] = vw / 3 - 2 * 1; t.draw_lo[k] = 1; t.draw_hi[k++] = vh - 1; }
        t.agent_angle = 0.0f;
    } else {
        const bool heavy = cfg.heavy != 0;
        const float dense = (float)(heavy ? 20.0 : 1.56);
        const double vw = 1440 / 560.0, vh = 810 / 560.0;
        for (int b = 0; b < t.n_blocks; ++b) {
            FixSpec fx[2]; int n;
            if (b == 0) { fx[0] = box_fix(0.1f, 0.1f, 0.0f, -0.1f, dense, 0.01f); fx[1] = box_fix(0.3f, 0.1f, 0.0f, 0.1f, dense, 0.01f); n = 2; }
            else if (b == 1) { fx[0] = box_fix(0.1f, 0.1f, 0.1f, 0.05f, dense, 0.01f); fx[1] = box_fix(0.1f, 0.2f, -0.1f, -0.05f, dense, 0.01f); n = 2; }
            else { std::memset(&fx[0], 0, sizeof(FixSpec)); poly_box(fx[0].shape, 0.1f, 0.2f); fx[0].density = dense; fx[0].friction = 0.01f; n = 1; }
            add_body(t, b, nfix, fx, n, true, 5.0f);
            save_vertices(t, b, fx, n);
            t.block_px[b] = vw / 2;
            t.block_py[b] = vh / 2 + (t.n_blocks == 3 ? (b == 1 ? 0.4 : (b == 2 ? -0.4 : 0.0)) : 0.0);
        }
        V2 poly[8] = {{-0.039f, -0.095f}, {0.039f, -0.095f}, {0.095f, -0.039f}, {0.095f, 0.039f},
                      {0.039f, 0.095f}, {-0.039f, 0.095f}, {-0.095f, 0.039f}, {-0.095f, -0.039f}};
        FixSpec af[3]; std::memset(af, 0, sizeof(af));
        poly_set(af[0].shape, poly, 8); af[0].density = 17.3f; af[0].friction = 0.01f;
        poly_box_oriented(af[1].shape, 0.005f, 0.05f, v2(0.06f, 0.0f), 0.0f); af[1].density = 0.0f; af[1].friction = 0.01f;
        poly_box_oriented(af[2].shape, 0.005f, 0.05f, v2(-0.06f, 0.0f), 0.0f); af[2].density = 0.0f; af[2].friction = 0.01f;
        for (int i = 0; i < t.n_agents; ++i) add_body(t, t.n_blocks + i, nfix, af, 3, true, 5.0f);
        const double bx[4] = {0, 1, 0.5, 0.5}, by[4] = {0.5, 0.5, 0, 1};
        for (int w = 0; w < 4; ++w) {
            FixSpec wf; std::memset(&wf, 0, sizeof(wf));
            poly_box(wf.shape, (float)(w < 2 ? 0.1 : vw), (float)(w < 2 ? vh : 0.1)); wf.density = 0.0f; wf.friction = 0.2f;
            int b = t.n_dyn + w;
            add_body(t, b, nfix, &wf, 1, false, 0.0f);
            t.wall_px[w] = (float)(vw * bx[w]); t.wall_py[w] = (float)(vh * by[w]);
        }
        t.agent_angle = (float)(3.0 / 2.0 * PI);
        int k = 0;
        for (int b = 0; b < t.n_blocks; ++b) { t.draw_lo[k] = 0.0; t.draw_hi[k++] = 2 * PI; }
        const double xr[2] = {0.3, vw / 3 - 0.3}, yr[2] = {0.3, vh - 0.3};
        for (int i = 0; i < t.n_agents; ++i) { t.draw_lo[k] = xr[0]; t.draw_hi[k++] = xr[1]; t.draw_lo[k] = yr[0]; t.draw_hi[k++] = yr[1]; }
        t.draw_lo[k] = vw * 2 / 3 + 0.4; t.draw_hi[k++] = vw - 0.4;
        t.draw_lo[k] = 0.4; t.draw_hi[k++] = vh - 0.4;
        if (t.n_blocks == 3) {   // build-defined square: offsets (world m) of L and I goals relative to the T goal
            t.goal_off[1][0] = -2.0 / 3.0 * 0.2; t.goal_off[1][1] = (-2.0 / 3.0 - 0.75) * 0.2; t.goal_off[1][2] = 0.5 * PI;
            t.goal_off[2][0] = 1.0 * 0.2; t.goal_off[2][1] = (-0.5 - 0.75) * 0.2; t.goal_off[2][2] = 0.0;
        }
    }
    t.n_fix = nfix;
    // obs layouts: multi_robot_puzzle_00.py:188-200 (4 per agent, block 4 + its vertices),
    // _02.py:178-188 (9 per agent, 4 + vertices per block, contact weight), core.py:121-132 (v3:
    // 4 per agent, block 3 + vertices)
    int nv = 0;
    for (int b = 0; b < nb; ++b) nv += 2 * t.nverts[b];
    t.obs_dim = cfg.version == 0 ? 4 * na + 4 + nv : (cfg.version == 3 ? 4 * na + 3 + nv : 9 * na + 4 * nb + nv + 1);
    return true;
}

void default_params(int env_id, EnvParams& p) {
    if (env_id < 0 || env_id >= N_ENVS || ENV_CFG[env_id].version != 2) {   // set_reward_params defaults multi_robot_puzzle_00.py:231-239, core.py:149-155
        p.w_dAgent = 10; p.w_agentDist = 0.1; p.w_dBlock = 50; p.w_blkDist = 0.025; p.scaled_epsilon = 25.0;
    } else {            // multi_robot_puzzle_02.py:216-225, EPSILON :58
        p.w_dAgent = 10; p.w_agentDist = 0.25; p.w_dBlock = 25; p.w_blkDist = 0.1; p.scaled_epsilon = 0.1;
    }
    // update_params(timestep=0, decay=1) values; the reference leaves these undefined until called
    p.shaped_bounds = 1000.0; p.shaped_blk_bounds = 100.0; p.shaped_puzzle = 10000.0;
    p.puzzle_complete = 100.0;
    p.frameskip = 1;   // the registered ids and the low-dim v0 obs step the world once (multi_robot_puzzle_00.py:161-162)
    p.pad = 0;
}

}  // namespace mrp
