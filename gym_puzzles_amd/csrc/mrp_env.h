// mrp_env.h -- env-level logic of one lane on top of World<ENV>: reset (destroy + rebuild
// + the reference's extra random-action step), action application, distances,
// observation, reward, done.  Python float64 semantics of the reference are reproduced
// in double precision (numpy 1.x scalar promotion; CPython float ** and %).
#pragma once
#include "mrp_world.h"

namespace mrp {

// Python float % (CPython float_rem / numpy npy_remainder): sign of the divisor
__device__ __forceinline__ double py_mod(double vx, double wx) {
    double mod = fmod(vx, wx);
    if (mod != 0.0) { if ((wx < 0) != (mod < 0)) mod += wx; }
    else mod = copysign(0.0, wx);
    return mod;
}
// distance() (multi_robot_puzzle_00.py:130-132): ((a-b)**2 + (c-d)**2) ** 0.5.  Known divergence: CPython's
// `**` calls glibc pow, which is not correctly rounded; the multiply and sqrt here are.  The two differ
// in the last bit of the float64 distance for rare inputs (the CPU oracle keeps pow, its libm_pow;
// the seed-11 / step-58 case is pinned in tests/test_v2_env_layer.py::test_distance_pow_semantics_known_case,
// where both round to the same float32).  The float32 obs and the done thresholds compare bit for bit
// in tests/test_gpu.py, which notes where a 1-ulp float64 difference could surface.
__device__ __forceinline__ double py_distance(double ax, double ay, double bx, double by) {
    double dx = ax - bx, dy = ay - by;
    double x = dx * dx, y = dy * dy;
    return sqrt(x + y);
}

constexpr double PY_PI = 3.141592653589793;
constexpr double TWO_PI = 6.283185307179586;

template <int ENV> struct Env : World<ENV> {
    using W = World<ENV>;
    using D = Dims<ENV>;
    using W::S; using W::T; using W::P; using W::sh; using W::tid;
    static constexpr int NA = D::NA, NB = D::NB, ND = W::ND, NF = D::NF;

    __device__ __forceinline__ Env(typename W::SH& s, const EnvTables& t, const EnvParams& p, int thread) : W(s, t, p, thread) {}

    __device__ __forceinline__ void init_empty_world() {   // fresh b2World (Box2D.b2World(gravity=(0,0), doSleep=False))
        constexpr int TN = W::LS::TN;
        for (int i = 0; i < TN; ++i) { S.tpar[i] = i + 1 < TN ? i + 1 : NULLN; S.th[i] = -1; S.tud[i] = -1; S.tc1[i] = NULLN; S.tc2[i] = NULLN; }
        S.root = NULLN; S.freeList = 0; S.nodeCount = 0; S.moveCount = 0;
        S.cHead = NULLN; S.cFree = 0; S.cCount = 0; S.cHW = 0;
        for (int c = 0; c < D::CMAX; ++c) S.cnext[c] = c + 1 < D::CMAX ? c + 1 : NULLN;
        S.inv_dt0 = 0.0f; S.newFixture = 0; S.haveBodies = 0; S.episode = 0; S.stepCounter = 0;
        S.elapsed = 0; S.blks_in_place = 0; S.prev_blks_in_place = 0; S.wall_contact = 0;
        S.toiEvents = 0; S.posIters = 0; S.touching = 0; S.nonfinite = 0;
    }

    // _destroy (multi_robot_puzzle_00.py:218-229): blocks, walls, agents; each body's proxies
    // in fixture-list order (newest first).  The listener is detached, so no End events.
    // v3 (core.py:246-262): boundary, goal block, agents.
    __device__ __forceinline__ void destroy_bodies() {
        if (!S.haveBodies) return;
        S.cHead = NULLN; S.cFree = 0; S.cCount = 0;
        for (int c = 0; c < D::CMAX; ++c) S.cnext[c] = c + 1 < D::CMAX ? c + 1 : NULLN;
        if (D::V == 3) {
            for (int b = ND; b < ND + 4; ++b) for (int k = T.body_nfix[b] - 1; k >= 0; --k) this->destroy_proxy(T.body_fix0[b] + k);
            for (int b = 0; b < ND; ++b) for (int k = T.body_nfix[b] - 1; k >= 0; --k) this->destroy_proxy(T.body_fix0[b] + k);
            S.haveBodies = 0;
            return;
        }
        for (int b = 0; b < NB; ++b) for (int k = T.body_nfix[b] - 1; k >= 0; --k) this->destroy_proxy(T.body_fix0[b] + k);
        for (int b = ND; b < ND + 4; ++b) for (int k = T.body_nfix[b] - 1; k >= 0; --k) this->destroy_proxy(T.body_fix0[b] + k);
        for (int b = NB; b < ND; ++b) for (int k = T.body_nfix[b] - 1; k >= 0; --k) this->destroy_proxy(T.body_fix0[b] + k);
        S.haveBodies = 0;
    }

    __device__ __forceinline__ void create_dyn_body(int b, float px, float py, float angle) {
        Rot q = rot(angle);
        S.xpx[b] = px; S.xpy[b] = py; S.xs[b] = q.s; S.xc[b] = q.c;
        V2 c = v2(px, py);
        if (T.body_reset_mass[b]) {
            Xf x; x.p = v2(px, py); x.q = q;
            c = mul_xv(x, v2(T.lcx[b], T.lcy[b]));   // ResetMassData: c0 = c = xf * localCenter
        }
        S.cx[b] = c.x; S.cy[b] = c.y; S.c0x[b] = c.x; S.c0y[b] = c.y;
        S.a[b] = angle; S.a0[b] = angle; S.alpha0[b] = 0.0f;
        S.vx[b] = 0.0f; S.vy[b] = 0.0f; S.w[b] = 0.0f; S.fx[b] = 0.0f; S.fy[b] = 0.0f; S.tq[b] = 0.0f;
        Xf x = this->xf(b);
        for (int k = 0; k < T.body_nfix[b]; ++k) this->create_proxy(T.body_fix0[b] + k, x);
    }

    // _generate_blocks / _generate_agents / _generate_boundary (+ v2 _set_random_goal)
    __device__ __forceinline__ void create_bodies(const double* d) {
        int k = 0;
        if (D::V == 0 || D::V == 3) {   // v3: Block(init_x, init_y, init_angle) then Robots at angle 0
            create_dyn_body(0, (float)d[0], (float)d[1], (float)d[2]);
            k = 3;
            for (int i = 0; i < NA; ++i) { create_dyn_body(NB + i, (float)d[k], (float)d[k + 1], 0.0f); k += 2; }
            S.goal[0][0] = T.goal_x; S.goal[0][1] = T.goal_y; S.goal[0][2] = T.goal_a;
        } else {
            for (int b = 0; b < NB; ++b) create_dyn_body(b, (float)T.block_px[b], (float)T.block_py[b], (float)d[k++]);
            for (int i = 0; i < NA; ++i) { create_dyn_body(NB + i, (float)d[k], (float)d[k + 1], T.agent_angle); k += 2; }
            const double ratio = 560.0 / 1440;
            double gx = d[k], gy = d[k + 1];
            S.goal[0][0] = gx * ratio; S.goal[0][1] = gy * ratio; S.goal[0][2] = 0.0;
            for (int b = 1; b < NB; ++b) {
                S.goal[b][0] = (gx + T.goal_off[b][0]) * ratio; S.goal[b][1] = (gy + T.goal_off[b][1]) * ratio; S.goal[b][2] = T.goal_off[b][2];
            }
        }
        for (int w = 0; w < 4; ++w) {
            int b = ND + w;
            Xf x = this->xf(b);
            for (int kk = 0; kk < T.body_nfix[b]; ++kk) this->create_proxy(T.body_fix0[b] + kk, x);
        }
        for (int i = 0; i < NA; ++i) S.goal_contact[i] = 0;
        S.newFixture = 1;
        S.haveBodies = 1;
    }

    // _calculate_distance / _calculate_agent_distance
    __device__ __forceinline__ void calc_distances() {
        if (D::V == 3) {   // the distances _get_obs stores (core.py:307-343), normalised poses
            double bx, by; norm_pose(0, bx, by);
            for (int i = 0; i < NA; ++i) {
                double ax, ay; norm_pose(NB + i, ax, ay);
                S.agent_dist[i] = py_distance(ax, ay, bx, by);
            }
            S.block_distance[0] = py_distance(bx, by, (S.goal[0][0] - 320.0) / 320.0, (S.goal[0][1] - 240.0) / 320.0);
        } else if (D::V == 0) {
            for (int b = 0; b < NB; ++b) {
                float sx = S.cx[b] * 30.0f, sy = S.cy[b] * 30.0f;   // b2Vec2 * SCALE (float32)
                S.block_distance[b] = py_distance(sx, sy, S.goal[b][0], S.goal[b][1]);
            }
            float bsx = S.cx[0] * 30.0f, bsy = S.cy[0] * 30.0f;
            for (int i = 0; i < NA; ++i) {
                float ax = S.cx[NB + i] * 30.0f, ay = S.cy[NB + i] * 30.0f;
                S.agent_dist[i] = py_distance(ax, ay, bsx, bsy);
            }
        } else {
            const double ratio = 560.0 / 1440;
            for (int b = 0; b < NB; ++b)
                S.block_distance[b] = py_distance((double)S.cx[b] * ratio, (double)S.cy[b] * ratio, S.goal[b][0], S.goal[b][1]);
            for (int i = 0; i < NA; ++i)
                S.agent_dist[i] = py_distance((double)S.cx[NB + i] * ratio, (double)S.cy[NB + i] * ratio, (double)S.cx[0] * ratio, (double)S.cy[0] * ratio);
        }
    }

    // RobotPuzzleBase._get_norm_pose (core.py:289-295): (x - ws) / ws, (y - hs) / ws
    __device__ __forceinline__ void norm_pose(int b, double& x, double& y) const {
        const double ws = 640 / 30.0 / 2, hs = 480 / 30.0 / 2;
        x = ((double)S.cx[b] - ws) / ws;
        y = ((double)S.cy[b] - hs) / ws;
    }
    __device__ __forceinline__ void unit_vector(int a, int b, double& ux, double& uy) const {   // unitVector :134-138
        double Ax = S.cx[a], Ay = S.cy[a], Bx = S.cx[b], By = S.cy[b];
        double dx = fabs(Bx - Ax), dy = fabs(By - Ay);
        double denom = dy > dx ? dy : dx;
        ux = (Bx - Ax) / denom; uy = (By - Ay) / denom;
    }
    __device__ __forceinline__ void apply_force(int b, V2 f, V2 point) {   // b2Body::ApplyForce
        S.fx[b] = S.fx[b] + f.x; S.fy[b] = S.fy[b] + f.y;
        S.tq[b] += vcross(vsub(point, v2(S.cx[b], S.cy[b])), f);
    }

    __device__ __forceinline__ void apply_actions(const float* act) {
        if (D::V == 0 || D::V == 3) {   // multi_robot_puzzle_00.py:415-424; v3 core.py:355-364 + robot.py:65-68
            const double SPEED = D::V == 3 ? 5.0 : 10.0 / 30.0 * 4;
            for (int i = 0; i < NA; ++i) {
                int ag = NB + i;
                float x = act[3 * i], y = act[3 * i + 1], turn = act[3 * i + 2];
                S.vx[ag] = (float)((double)x * SPEED); S.vy[ag] = (float)((double)y * SPEED);
                S.w[ag] = turn;
                double force = pow(1.1, -S.agent_dist[i]);
                double ux, uy; unit_vector(ag, 0, ux, uy);
                apply_force(0, v2((float)(force * ux), (float)(force * uy)), v2(S.cx[0], S.cy[0]));
            }
        } else {           // multi_robot_puzzle_02.py:446-474
            for (int i = 0; i < NA; ++i) {
                int ag = NB + i;
                float turn = act[2 * i], vel = act[2 * i + 1];
                Rot q; q.s = S.xs[ag]; q.c = S.xc[ag];
                V2 f = mul_rv(q, v2(0.0f, 1.0f));
                Xf x = this->xf(ag);
                V2 p = mul_xv(x, v2(0.0f, 2.0f));
                double fx = (double)f.x * (double)vel * 0.75, fy = (double)f.y * (double)vel * 0.75;
                apply_force(ag, v2((float)fx, (float)fy), p);
                // updateFriction :116-122 (pybox2d b2Vec2 arithmetic is float32)
                V2 n = mul_rv(q, v2(1.0f, 0.0f));
                float dlat = n.x * S.vx[ag] + n.y * S.vy[ag];
                V2 lat = v2(n.x * dlat, n.y * dlat);
                V2 nl = v2(-lat.x, -lat.y);
                float m = T.mass[ag];
                V2 imp = v2(nl.x * m, nl.y * m);
                S.vx[ag] = S.vx[ag] + T.invMass[ag] * imp.x; S.vy[ag] = S.vy[ag] + T.invMass[ag] * imp.y;
                S.w[ag] += T.invI[ag] * vcross(vsub(v2(S.cx[ag], S.cy[ag]), v2(S.cx[ag], S.cy[ag])), imp);
                float inertia = T.I[ag] + T.mass[ag] * vdot(v2(T.lcx[ag], T.lcy[ag]), v2(T.lcx[ag], T.lcy[ag]));
                S.w[ag] += T.invI[ag] * (float)(0.1 * (double)inertia * (double)S.w[ag]);
                double torque = (double)fabsf(turn) * 0.0005;
                double tsel = turn;
                if (fabs((double)vel) < 0.1) tsel = 0.0;
                if (tsel < 0) S.tq[ag] += (float)torque;
                else if (tsel > 0) S.tq[ag] += (float)(-torque);
                else S.tq[ag] += 0.0f;
                double force = pow(10.0, -S.agent_dist[i]);
                force /= 50;
                double ux, uy; unit_vector(ag, 0, ux, uy);
                apply_force(0, v2((float)(force * ux), (float)(force * uy)), v2(S.cx[0], S.cy[0]));
            }
        }
    }

    // observation :442-472 / _02.py:494-532, reward + done :475-521 / _02.py:535-584
    __device__ __forceinline__ void obs_reward(const double* prevA, const double* prevB, float* obs, double& reward_out, int& done_out, int& kind_out) {
        int k = 0;
        bool in_place[NB];
        double reward = 0.0; int done = 0, kind = 0;
        if (D::V == 3) {   // _get_obs core.py:297-350, step core.py:369-414
            const double ws = 640 / 30.0 / 2, hs = 480 / 30.0 / 2;
            double bx, by; norm_pose(0, bx, by);
            const double brot = py_mod((double)S.a[0], TWO_PI);
            for (int i = 0; i < NA; ++i) {
                double ax, ay; norm_pose(NB + i, ax, ay);
                obs[k++] = (float)(bx - ax); obs[k++] = (float)(by - ay);
                obs[k++] = (float)py_mod((double)S.a[NB + i], TWO_PI);
                obs[k++] = S.goal_contact[i] ? 1.0f : 0.0f;
            }
            const double gx = (S.goal[0][0] - 320.0) / 320.0, gy = (S.goal[0][1] - 240.0) / 320.0;
            obs[k++] = (float)(gx - bx); obs[k++] = (float)(gy - by); obs[k++] = (float)(py_mod(S.goal[0][2], TWO_PI) - brot);
            Xf xb = this->xf(0);
            for (int j = 0; j < T.nverts[0]; ++j) {   // Block.get_vertices(norm_fn) blocks.py:118-123
                V2 wp = mul_xv(xb, T.verts[0][j]);
                obs[k++] = (float)(((double)wp.x - ws) / ws); obs[k++] = (float)(((double)wp.y - hs) / ws);
            }
            const bool in_place0 = S.block_distance[0] <= 25.0 / 640 * 2;
            double deltaDist = prevB[0] - S.block_distance[0];
            reward += deltaDist * P.w_dBlock;
            reward -= P.w_blkDist * S.block_distance[0];
            for (int i = 0; i < NA; ++i) {
                double deltaAgent = prevA[i] - S.agent_dist[i];
                reward += deltaAgent * P.w_dAgent / 4.;
                reward -= P.w_agentDist * S.agent_dist[i] / 4.;
                if (S.goal_contact[i]) reward += 0.25;
            }
            if (in_place0) { done = 1; kind = 1; reward += P.puzzle_complete; }
        } else if (D::V == 0) {
            for (int i = 0; i < NA; ++i) {
                double x = S.cx[0], y = S.cy[0];
                obs[k++] = (float)((double)S.cx[NB + i] * 30.0 - x * 30.0);
                obs[k++] = (float)((double)S.cy[NB + i] * 30.0 - y * 30.0);
                obs[k++] = (float)S.agent_dist[i];
                obs[k++] = S.goal_contact[i] ? 1.0f : 0.0f;
            }
            for (int b = 0; b < NB; ++b) {
                double x = S.cx[b], y = S.cy[b];
                double angle = py_mod((double)S.a[b], TWO_PI);
                double fx = S.goal[b][0], fy = S.goal[b][1], fangle = S.goal[b][2];
                x *= 30.0; y *= 30.0;
                double a_diff = py_mod(fangle, TWO_PI) - angle;
                in_place[b] = !(fabs(fx - x) > 25.0) && !(fabs(fy - y) > 25.0);
                obs[k++] = (float)(x - fx); obs[k++] = (float)(y - fy); obs[k++] = (float)a_diff;
                obs[k++] = (float)py_distance(x, y, fx, fy);
                Xf xb = this->xf(b);
                for (int j = 0; j < T.nverts[b]; ++j) {
                    V2 wp = mul_xv(xb, T.verts[b][j]);
                    obs[k++] = (float)((double)wp.x * 30.0); obs[k++] = (float)((double)wp.y * 30.0);
                }
            }
            double deltaDist = prevB[0] - S.block_distance[0];
            reward += deltaDist * P.w_dBlock * 1.0 / 4.;
            reward -= P.w_blkDist * S.block_distance[0] * 1.0 / 4.;
            for (int i = 0; i < NA; ++i) {
                double deltaAgent = prevA[i] - S.agent_dist[i];
                reward += deltaAgent * P.w_dAgent * 1.0 / 4.;
                reward -= P.w_agentDist * S.agent_dist[i] * 1.0 / 4.;
                if (S.goal_contact[i]) reward += 0.25;
            }
            S.prev_blks_in_place = S.blks_in_place;
            S.blks_in_place = 0;
            for (int b = 0; b < NB; ++b) if (in_place[b]) S.blks_in_place += 1;
            reward += (double)((S.blks_in_place - S.prev_blks_in_place) * 10);
            if (S.blks_in_place == 1) { done = 1; kind = 1; reward += 10000; }
        } else {
            const double ratio = 560.0 / 1440;
            for (int i = 0; i < NA; ++i) {
                int ag = NB + i;
                double aX = (double)S.cx[ag] * ratio, aY = (double)S.cy[ag] * ratio;
                double theta = py_mod((double)S.a[ag], TWO_PI);
                double nt = theta <= PY_PI ? -theta / PY_PI : (TWO_PI - theta) / PY_PI;
                double bX = (double)S.cx[0] * ratio, bY = (double)S.cy[0] * ratio;
                obs[k++] = (float)aX; obs[k++] = (float)aY; obs[k++] = (float)nt;
                obs[k++] = (float)(aX - bX); obs[k++] = (float)(aY - bY);
                obs[k++] = S.vx[ag]; obs[k++] = S.vy[ag]; obs[k++] = S.w[ag];
                obs[k++] = (float)S.agent_dist[i];
            }
            for (int b = 0; b < NB; ++b) {
                double x = (double)S.cx[b] * ratio, y = (double)S.cy[b] * ratio;
                double angle = py_mod((double)S.a[b], TWO_PI);
                double fx = S.goal[b][0], fy = S.goal[b][1], fangle = S.goal[b][2];
                double a_diff = py_mod(fangle, TWO_PI) - angle;
                a_diff /= PY_PI;
                in_place[b] = !(fabs(fx - x) > P.scaled_epsilon) && !(fabs(fy - y) > P.scaled_epsilon);
                obs[k++] = (float)(x - fx); obs[k++] = (float)(y - fy); obs[k++] = (float)a_diff;
                obs[k++] = (float)py_distance(x, y, fx, fy);
                Xf xb = this->xf(b);
                for (int j = 0; j < T.nverts[b]; ++j) {
                    V2 wp = mul_xv(xb, T.verts[b][j]);
                    obs[k++] = (float)((double)wp.x * ratio); obs[k++] = (float)((double)wp.y * ratio);
                }
            }
            obs[k++] = (float)P.scaled_epsilon;
            double deltaDist = prevB[0] - S.block_distance[0];
            reward += deltaDist * P.w_dBlock;
            reward -= P.w_blkDist * S.block_distance[0];
            for (int i = 0; i < NA; ++i) {
                double deltaAgent = prevA[i] - S.agent_dist[i];
                reward += deltaAgent * P.w_dAgent;
                reward -= P.w_agentDist * S.agent_dist[i];
            }
            const double vw = 1440 / 560.0, vh = 810 / 560.0;
            bool agt_oob = false, blk_oob = false;
            for (int i = 0; i < NA && !agt_oob; ++i) {
                double x = S.cx[NB + i], y = S.cy[NB + i];
                if (x < 0.1 || x > (vw - 0.1)) agt_oob = true;
                else if (y < 0.1 || y > (vh - 0.1)) agt_oob = true;
            }
            for (int b = 0; b < NB && !blk_oob; ++b) {
                double x = S.cx[b], y = S.cy[b];
                if (x < 0.1 || x > (vw - 0.1)) blk_oob = true;
                else if (y < 0.1 || y > (vh - 0.1)) blk_oob = true;
            }
            if (agt_oob) { done = 1; kind = 2; reward -= P.shaped_bounds; }
            else if (blk_oob) { done = 1; kind = 3; reward -= P.shaped_blk_bounds; }
            else {
                S.prev_blks_in_place = S.blks_in_place;
                S.blks_in_place = 0;
                for (int b = 0; b < NB; ++b) if (in_place[b]) S.blks_in_place += 1;
                int num_in_contact = 0;
                for (int i = 0; i < NA; ++i) if (S.goal_contact[i]) num_in_contact += 1;
                if (S.blks_in_place == NB) { done = 1; kind = 1; reward += P.shaped_puzzle * ((double)num_in_contact / (double)NA); }
            }
        }
        reward_out = reward; done_out = done; kind_out = kind;
    }

    // one env step (cooperative: every thread of the wave calls it); reads sh.act, writes
    // sh.obs / sh.reward / sh.done / sh.kind
    __device__ __forceinline__ void env_step_coop() {
        if (tid == 0) apply_actions(sh.act);
        __syncthreads();
        MRP_STAMP(1);
        // for _ in range(self.frameskip): world.Step(...) (multi_robot_puzzle_02.py:476-478); the
        // applied forces are cleared by the first Step, as Box2D's autoClearForces does
        const int fs = P.frameskip > 1 ? P.frameskip : 1;
        for (int f = 0; f < fs; ++f) this->world_step_coop();
        if (tid == 0) {
            double prevA[NA], prevB[NB];
            for (int i = 0; i < NA; ++i) prevA[i] = S.agent_dist[i];
            for (int b = 0; b < NB; ++b) prevB[b] = S.block_distance[b];
            calc_distances();
            obs_reward(prevA, prevB, sh.obs, sh.reward, sh.done, sh.kind);
        }
        __syncthreads();
        MRP_STAMP(7);
    }

    // reset(): destroy + rebuild from sh.draws, then the reference's step with sh.act
    __device__ __forceinline__ void env_reset_coop() {
        {   // the contact slots used since the last reset back to their initial contents (destroy_bodies
            // rebuilds the free chain), so every slot is initial again (LaneState::cHW)
            using LS = typename W::LS;
            const int hw = S.cHW;
            typedef uint32_t __attribute__((__may_alias__)) aw_t;
            aw_t* w = reinterpret_cast<aw_t*>(S.cprev);   // cprev .. mid[1]: NCA - 1 arrays
            for (int i = tid; i < (LS::NCA - 1) * D::CMAX; i += 64)   // the wave
                if (i % D::CMAX < hw) w[i] = 0u;
        }
        __syncthreads();
        if (tid == 0) {
            S.cHW = 0;
            destroy_bodies();
            create_bodies(sh.draws);
            calc_distances();
        }
        __syncthreads();
        env_step_coop();
    }
};

}  // namespace mrp
