// slo_pg.hip — pose-graph back end (host code).
//
// Replaces the GTSAM iSAM2 graph mapOptimization keeps over its key poses:
//   - prior on key pose 0, variances (1e-6,1e-6,1e-6, 1e-8,1e-8,1e-6)      MO:365-368, 1541-1546
//   - odometry BetweenFactor(k-1, k, transformLast.between(transformAftMapped)) MO:1547-1555
//   - loop BetweenFactor(latest, history, poseFrom.between(poseTo)) with a
//     Cauchy(1) robust model on variances 0.5                               MO:985-997, 1038-1046, 1083-1091
//   - latestEstimate → transformAftMapped / transformLast                    MO:1566-1611
//   - correctPoses: every key pose from the current estimate                 MO:1642-1664
// GTSAM is absent from the image, so the solve is a batch Levenberg-Marquardt
// to convergence of the same factor graph (the fixed point iSAM2's
// incremental Gauss-Newton tracks).  Conventions follow GTSAM 4 with
// Pose3/Rot3 expmap charts: tangent order [rot(3), trans(3)], retract
// T*Exp(d), between error Log(Z^-1 * Ti^-1 * Tj), prior error Log(Z^-1 * T0),
// Cauchy weight 1/(1 + |e_w|^2/k^2) on the whole whitened factor error.
// The graph is a chain plus a few loop edges, so the normal matrix is stored
// as a skyline (per-row envelope) and factored in place: a loop (i, j) adds
// only the rows of pose j out to pose i, and Cholesky fill stays inside the
// envelope.  Scalar host work: a few hundred poses per map, no device launch.
#include "../../include/slo_abi.h"

#include <cmath>
#include <cstring>
#include <new>
#include <string>
#include <vector>

namespace {

struct Pose {
    double R[9];  // row-major
    double t[3];
};

void mat_mul(const double* A, const double* B, double* C) {
    for (int r = 0; r < 3; ++r)
        for (int c = 0; c < 3; ++c) C[r * 3 + c] = A[r * 3] * B[c] + A[r * 3 + 1] * B[3 + c] + A[r * 3 + 2] * B[6 + c];
}

Pose compose(const Pose& a, const Pose& b) {
    Pose o;
    mat_mul(a.R, b.R, o.R);
    for (int r = 0; r < 3; ++r) o.t[r] = a.R[r * 3] * b.t[0] + a.R[r * 3 + 1] * b.t[1] + a.R[r * 3 + 2] * b.t[2] + a.t[r];
    return o;
}

Pose inverse(const Pose& a) {
    Pose o;
    for (int r = 0; r < 3; ++r)
        for (int c = 0; c < 3; ++c) o.R[r * 3 + c] = a.R[c * 3 + r];
    for (int r = 0; r < 3; ++r) o.t[r] = -(o.R[r * 3] * a.t[0] + o.R[r * 3 + 1] * a.t[1] + o.R[r * 3 + 2] * a.t[2]);
    return o;
}

// Rot3::RzRyRx(x, y, z) = Rz(z) * Ry(y) * Rx(x)
Pose pose_rzryrx(double x, double y, double z, double tx, double ty, double tz) {
    double cx = std::cos(x), sx = std::sin(x), cy = std::cos(y), sy = std::sin(y), cz = std::cos(z), sz = std::sin(z);
    Pose p;
    double Rx[9] = {1, 0, 0, 0, cx, -sx, 0, sx, cx};
    double Ry[9] = {cy, 0, sy, 0, 1, 0, -sy, 0, cy};
    double Rz[9] = {cz, -sz, 0, sz, cz, 0, 0, 0, 1};
    double T[9];
    mat_mul(Rz, Ry, T);
    mat_mul(T, Rx, p.R);
    p.t[0] = tx; p.t[1] = ty; p.t[2] = tz;
    return p;
}

// Rot3::xyz(): roll (about x), pitch (about y), yaw (about z) of R = Rz Ry Rx
void rot_xyz(const double* R, double* xyz) {
    xyz[0] = std::atan2(R[7], R[8]);
    xyz[1] = std::atan2(-R[6], std::sqrt(R[7] * R[7] + R[8] * R[8]));
    xyz[2] = std::atan2(R[3], R[0]);
}

void hat(const double* w, double* W) {
    W[0] = 0;     W[1] = -w[2]; W[2] = w[1];
    W[3] = w[2];  W[4] = 0;     W[5] = -w[0];
    W[6] = -w[1]; W[7] = w[0];  W[8] = 0;
}

Pose se3_exp(const double* d) {
    const double* w = d;
    const double* v = d + 3;
    double th2 = w[0] * w[0] + w[1] * w[1] + w[2] * w[2], th = std::sqrt(th2);
    double A, B, C;  // sin/th, (1-cos)/th^2, (th-sin)/th^3
    if (th < 1e-5) {
        A = 1 - th2 / 6; B = 0.5 - th2 / 24; C = 1.0 / 6 - th2 / 120;
    } else {
        A = std::sin(th) / th; B = (1 - std::cos(th)) / th2; C = (th - std::sin(th)) / (th2 * th);
    }
    double W[9], W2[9];
    hat(w, W);
    mat_mul(W, W, W2);
    Pose p;
    for (int i = 0; i < 9; ++i) {
        double I = (i % 4 == 0) ? 1.0 : 0.0;
        p.R[i] = I + A * W[i] + B * W2[i];
    }
    double V[9];
    for (int i = 0; i < 9; ++i) V[i] = ((i % 4 == 0) ? 1.0 : 0.0) + B * W[i] + C * W2[i];
    for (int r = 0; r < 3; ++r) p.t[r] = V[r * 3] * v[0] + V[r * 3 + 1] * v[1] + V[r * 3 + 2] * v[2];
    return p;
}

void so3_log(const double* R, double* w) {
    // theta = atan2(|axis sin|, cos): acos of (tr - 1) / 2 loses half the
    // digits at the small angles the stiff odometry factors live at (an angle
    // of 1e-7 rad would carry a 1 % error), which stalls the solve
    double tr = R[0] + R[4] + R[8];
    double c = 0.5 * (tr - 1);
    const double v[3] = {0.5 * (R[7] - R[5]), 0.5 * (R[2] - R[6]), 0.5 * (R[3] - R[1])};
    const double sn = std::sqrt(v[0] * v[0] + v[1] * v[1] + v[2] * v[2]);
    double th = std::atan2(sn, c);
    if (th > M_PI - 1e-4) {  // near pi: axis from the largest diagonal of (R + I)/2
        int k = (R[0] >= R[4] && R[0] >= R[8]) ? 0 : (R[4] >= R[8] ? 1 : 2);
        double a[3];
        double s = std::sqrt(std::fmax(0.0, 0.5 * (R[k * 4] + 1)));
        for (int i = 0; i < 3; ++i) a[i] = (i == k) ? s : 0.5 * R[i * 3 + k] / s;
        double sgn = (R[7] - R[5]) * a[0] + (R[2] - R[6]) * a[1] + (R[3] - R[1]) * a[2];  // antisymmetric part
        if (sgn < 0) for (int i = 0; i < 3; ++i) a[i] = -a[i];
        double n = std::sqrt(a[0] * a[0] + a[1] * a[1] + a[2] * a[2]);
        for (int i = 0; i < 3; ++i) w[i] = th * a[i] / n;
        return;
    }
    const double f = (sn < 1e-12) ? 1.0 + th * th / 6 : th / sn;   // theta / sin(theta)
    w[0] = f * v[0];
    w[1] = f * v[1];
    w[2] = f * v[2];
}

void se3_log(const Pose& p, double* d) {
    double* w = d;
    so3_log(p.R, w);
    double th2 = w[0] * w[0] + w[1] * w[1] + w[2] * w[2], th = std::sqrt(th2);
    double D;  // V^-1 = I - W/2 + D W^2
    if (th < 1e-5) D = 1.0 / 12 + th2 / 720;
    else D = (1 - th * std::sin(th) / (2 * (1 - std::cos(th)))) / th2;
    double W[9], W2[9];
    hat(w, W);
    mat_mul(W, W, W2);
    for (int r = 0; r < 3; ++r) {
        double s = p.t[r];
        for (int c = 0; c < 3; ++c) s += (-0.5 * W[r * 3 + c] + D * W2[r * 3 + c]) * p.t[c];
        d[3 + r] = s;
    }
}

struct Factor {
    int i, j;      // j < 0: prior on i
    Pose Zinv;     // inverse measurement
    double sinv[6];
    bool robust;
};

}  // namespace

struct slo_pg {
    std::vector<Pose> est;
    std::vector<Factor> fac;
    double last[6];  // transformLast (LeGO order rx ry rz tx ty tz, camera frame)
    std::string err;
};

namespace {

const double kOdoVar[6] = {1e-6, 1e-6, 1e-6, 1e-8, 1e-8, 1e-6};  // MO:366
const double kLoopVar = 0.5;                                        // MO:989

// transformTobeMapped order → Pose3(RzRyRx(t2, t0, t1), Point3(t5, t3, t4))  (MO:1543, 1550-1553)
Pose pose_from_transform(const double* t) { return pose_rzryrx(t[2], t[0], t[1], t[5], t[3], t[4]); }

void transform_from_pose(const Pose& p, double* t) {
    double xyz[3];
    rot_xyz(p.R, xyz);
    t[0] = xyz[1]; t[1] = xyz[2]; t[2] = xyz[0];  // MO:1602-1604
    t[3] = p.t[1]; t[4] = p.t[2]; t[5] = p.t[0];
}

void factor_error(const Factor& f, const std::vector<Pose>& x, double* e) {
    Pose h = (f.j < 0) ? x[f.i] : compose(inverse(x[f.i]), x[f.j]);
    se3_log(compose(f.Zinv, h), e);
    for (int k = 0; k < 6; ++k) e[k] *= f.sinv[k];
}

// robust weight and cost contribution of a whitened error
double factor_cost(const Factor& f, const double* e, double* wt) {
    double r2 = 0;
    for (int k = 0; k < 6; ++k) r2 += e[k] * e[k];
    if (!f.robust) { if (wt) *wt = 1; return 0.5 * r2; }
    if (wt) *wt = 1.0 / (1.0 + r2);  // Cauchy, k = 1
    return 0.5 * std::log1p(r2);
}

double total_cost(const slo_pg* g, const std::vector<Pose>& x) {
    double c = 0, e[6];
    for (const Factor& f : g->fac) { factor_error(f, x, e); c += factor_cost(f, e, nullptr); }
    return c;
}

// skyline (row envelope) symmetric matrix: row r holds columns first[r] .. r
struct Skyline {
    std::vector<int> first;
    std::vector<size_t> off;
    std::vector<double> v;
    double& at(int r, int c) { return v[off[r] + (c - first[r])]; }
    double get(int r, int c) const { return c < first[r] ? 0.0 : v[off[r] + (c - first[r])]; }
};

bool skyline_cholesky(Skyline& S, int n) {
    for (int r = 0; r < n; ++r) {
        for (int c = S.first[r]; c <= r; ++c) {
            int k0 = S.first[r] > S.first[c] ? S.first[r] : S.first[c];
            double s = S.at(r, c);
            const double* lr = &S.v[S.off[r] + (k0 - S.first[r])];
            const double* lc = &S.v[S.off[c] + (k0 - S.first[c])];
            for (int k = 0; k < c - k0; ++k) s -= lr[k] * lc[k];
            if (c == r) {
                if (!(s > 0)) return false;
                S.at(r, r) = std::sqrt(s);
            } else {
                S.at(r, c) = s / S.at(c, c);
            }
        }
    }
    return true;
}

void skyline_solve(const Skyline& L, int n, double* b) {
    for (int r = 0; r < n; ++r) {
        double s = b[r];
        for (int c = L.first[r]; c < r; ++c) s -= L.get(r, c) * b[c];
        b[r] = s / L.get(r, r);
    }
    for (int r = n - 1; r >= 0; --r) {
        b[r] /= L.get(r, r);
        double br = b[r];
        for (int c = L.first[r]; c < r; ++c) b[c] -= L.get(r, c) * br;
    }
}

// one linearisation: H (skyline), g = J^T W e, per-factor numeric Jacobians
// (central differences of the right-perturbed error, h = 1e-5)
void linearise(const slo_pg* g, const std::vector<Pose>& x, Skyline& H, std::vector<double>& b) {
    std::fill(H.v.begin(), H.v.end(), 0.0);
    std::fill(b.begin(), b.end(), 0.0);
    const double h = 1e-5;
    std::vector<Pose> xp = x;
    for (const Factor& f : g->fac) {
        double e[6], wt;
        factor_error(f, x, e);
        factor_cost(f, e, &wt);
        int blocks[2] = {f.i, f.j};
        int nb = f.j < 0 ? 1 : 2;
        double J[2][6][6];  // J[b][row][col]
        for (int bi = 0; bi < nb; ++bi) {
            int p = blocks[bi];
            for (int c = 0; c < 6; ++c) {
                double d[6] = {0, 0, 0, 0, 0, 0}, ep[6], em[6];
                d[c] = h;
                xp[p] = compose(x[p], se3_exp(d));
                factor_error(f, xp, ep);
                d[c] = -h;
                xp[p] = compose(x[p], se3_exp(d));
                factor_error(f, xp, em);
                xp[p] = x[p];
                for (int r = 0; r < 6; ++r) J[bi][r][c] = (ep[r] - em[r]) / (2 * h);
            }
        }
        for (int a = 0; a < nb; ++a) {
            for (int ra = 0; ra < 6; ++ra) {
                int R = 6 * blocks[a] + ra;
                double s = 0;
                for (int k = 0; k < 6; ++k) s += J[a][k][ra] * e[k];
                b[R] -= wt * s;
                for (int bb = 0; bb < nb; ++bb) {
                    for (int cb = 0; cb < 6; ++cb) {
                        int C = 6 * blocks[bb] + cb;
                        if (C > R) continue;
                        double t = 0;
                        for (int k = 0; k < 6; ++k) t += J[a][k][ra] * J[bb][k][cb];
                        H.at(R, C) += wt * t;
                    }
                }
            }
        }
    }
}

int fail(slo_pg* g, int code, const char* msg) {
    if (g) g->err = msg;
    return code;
}

// the entry points promise not to throw (C callers): an allocation failure
// inside becomes SLO_E_CAPACITY with the message kept
template <class F>
int guarded(slo_pg* g, const char* where, F&& f) {
    try {
        return f();
    } catch (const std::bad_alloc&) {
        try { if (g) g->err = std::string(where) + ": out of memory"; } catch (...) {}
        return SLO_E_CAPACITY;
    } catch (...) {
        try { if (g) g->err = std::string(where) + ": internal error"; } catch (...) {}
        return SLO_E_STATE;
    }
}

}  // namespace

extern "C" {

int slo_pg_create(slo_pg** out) {
    if (!out) return SLO_E_ARG;
    *out = new (std::nothrow) slo_pg();
    return *out ? SLO_OK : SLO_E_CAPACITY;
}

void slo_pg_destroy(slo_pg* g) { delete g; }

const char* slo_pg_last_error(slo_pg* g) { return g ? g->err.c_str() : "null graph"; }

int slo_pg_size(slo_pg* g) { return g ? (int)g->est.size() : SLO_E_ARG; }

int slo_pg_add_keyframe(slo_pg* g, const float transform[6], float transform_out[6], float key_pose6d[6]) {
    if (!g || !transform) return fail(g, SLO_E_ARG, "slo_pg_add_keyframe: null argument");
    return guarded(g, "slo_pg_add_keyframe", [&]() -> int {
    double t[6];
    for (int k = 0; k < 6; ++k) t[k] = transform[k];
    Factor f;
    for (int k = 0; k < 6; ++k) f.sinv[k] = 1.0 / std::sqrt(kOdoVar[k]);
    f.robust = false;
    if (g->est.empty()) {  // MO:1541-1546: prior at transformTobeMapped
        Pose p = pose_from_transform(t);
        f.i = 0; f.j = -1; f.Zinv = inverse(p);
        g->est.push_back(p);
        std::memcpy(g->last, t, sizeof t);
    } else {  // MO:1547-1555: between(transformLast, transformAftMapped)
        Pose from = pose_from_transform(g->last), to = pose_from_transform(t);
        Pose z = compose(inverse(from), to);
        int n = (int)g->est.size();
        f.i = n - 1; f.j = n; f.Zinv = inverse(z);
        // the new pose's only factor is this between: its optimum is est[n-1] * z
        g->est.push_back(compose(g->est[n - 1], z));
    }
    g->fac.push_back(f);
    double o[6];
    transform_from_pose(g->est.back(), o);
    if (g->est.size() > 1) std::memcpy(g->last, o, sizeof o);  // MO:1601-1611
    if (transform_out) for (int k = 0; k < 6; ++k) transform_out[k] = (float)(g->est.size() > 1 ? o[k] : t[k]);
    if (key_pose6d) {
        const Pose& p = g->est.back();
        double xyz[3];
        rot_xyz(p.R, xyz);
        // MO:1580-1593: x = t.y, y = t.z, z = t.x, roll = pitch(), pitch = yaw(), yaw = roll()
        key_pose6d[0] = (float)p.t[1]; key_pose6d[1] = (float)p.t[2]; key_pose6d[2] = (float)p.t[0];
        key_pose6d[3] = (float)xyz[1]; key_pose6d[4] = (float)xyz[2]; key_pose6d[5] = (float)xyz[0];
    }
    return SLO_OK;
    });
}

int slo_pg_add_loop(slo_pg* g, int from_id, int to_id, const float pose_from[6], const float pose_to[6]) {
    if (!g || !pose_from || !pose_to) return fail(g, SLO_E_ARG, "slo_pg_add_loop: null argument");
    int n = (int)g->est.size();
    if (from_id < 0 || to_id < 0 || from_id >= n || to_id >= n || from_id == to_id)
        return fail(g, SLO_E_ARG, "slo_pg_add_loop: key pose id out of range");
    return guarded(g, "slo_pg_add_loop", [&]() -> int {
    // Pose3(Rot3::RzRyRx(v0, v1, v2), Point3(v3, v4, v5)), as MO:1035-1037 / 1080-1082 build them
    Pose a = pose_rzryrx(pose_from[0], pose_from[1], pose_from[2], pose_from[3], pose_from[4], pose_from[5]);
    Pose b = pose_rzryrx(pose_to[0], pose_to[1], pose_to[2], pose_to[3], pose_to[4], pose_to[5]);
    Factor f;
    f.i = from_id; f.j = to_id;
    f.Zinv = inverse(compose(inverse(a), b));
    for (int k = 0; k < 6; ++k) f.sinv[k] = 1.0 / std::sqrt(kLoopVar);
    f.robust = true;
    g->fac.push_back(f);
    return SLO_OK;
    });
}

int slo_pg_optimize(slo_pg* g, int max_iters, int* iters_out, double* cost_out) {
    if (!g) return SLO_E_ARG;
    int n = (int)g->est.size(), N = 6 * n;
    if (n == 0) return fail(g, SLO_E_STATE, "slo_pg_optimize: empty graph");
    if (max_iters <= 0) max_iters = 100;
    return guarded(g, "slo_pg_optimize", [&]() -> int {
    // envelope: each pose's rows reach back to its lowest connected pose
    std::vector<int> lo(n);
    for (int p = 0; p < n; ++p) lo[p] = p;
    for (const Factor& f : g->fac)
        if (f.j >= 0) {
            int a = f.i < f.j ? f.i : f.j, b = f.i < f.j ? f.j : f.i;
            if (a < lo[b]) lo[b] = a;
        }
    Skyline H;
    H.first.resize(N);
    H.off.resize(N + 1);
    size_t off = 0;
    for (int r = 0; r < N; ++r) {
        H.first[r] = 6 * lo[r / 6];
        H.off[r] = off;
        off += (size_t)(r - H.first[r] + 1);
    }
    H.off[N] = off;
    H.v.assign(off, 0.0);
    Skyline L = H;
    std::vector<double> b(N), dx(N);
    std::vector<Pose> trial(n);
    double cost = total_cost(g, g->est), lambda = 1e-5;
    int it = 0;
    bool converged = false;
    for (; it < max_iters; ++it) {
        linearise(g, g->est, H, b);
        bool accepted = false;
        for (int tries = 0; tries < 12 && !accepted; ++tries) {
            L.v = H.v;
            for (int r = 0; r < N; ++r) L.at(r, r) += lambda * (H.get(r, r) > 1e-12 ? H.get(r, r) : 1e-12);
            if (!skyline_cholesky(L, N)) { lambda *= 10; continue; }
            dx = b;
            skyline_solve(L, N, dx.data());
            for (int p = 0; p < n; ++p) trial[p] = compose(g->est[p], se3_exp(&dx[6 * p]));
            double c = total_cost(g, trial);
            if (c <= cost) {
                double dec = cost - c;
                g->est.swap(trial);
                accepted = true;
                lambda = lambda > 1e-12 ? lambda * 0.1 : lambda;
                double old = cost;
                cost = c;
                if (dec <= 1e-12 * (old > 1e-300 ? old : 1e-300) || dec < 1e-18) { ++it; converged = true; goto done; }
            } else {
                lambda *= 10;
            }
        }
        if (!accepted) { converged = true; break; }  // no decrease at any damping: converged to rounding
    }
done:
    // transformLast is not touched here: the reference refreshes it only in
    // saveKeyFramesAndFactor (MO:1601-1611), so the next odometry factor is
    // measured from the pre-correction pose, as in the reference
    if (iters_out) *iters_out = it;
    if (cost_out) *cost_out = cost;
    if (!converged) {
        g->err = "slo_pg_optimize: max_iters reached before convergence";
        return SLO_NOT_CONVERGED;
    }
    return SLO_OK;
    });
}

// correctPoses (MO:1642-1664): cloudKeyPoses6D for every key pose, PointTypePose order x y z roll pitch yaw
int slo_pg_get_key_poses(slo_pg* g, float* out6, int cap) {
    if (!g || (!out6 && cap > 0)) return SLO_E_ARG;
    int n = (int)g->est.size();
    if (cap < n) return fail(g, SLO_E_CAPACITY, "slo_pg_get_key_poses: cap below graph size");
    for (int p = 0; p < n; ++p) {
        const Pose& q = g->est[p];
        double xyz[3];
        rot_xyz(q.R, xyz);
        float* o = out6 + 6 * p;
        o[0] = (float)q.t[1]; o[1] = (float)q.t[2]; o[2] = (float)q.t[0];
        o[3] = (float)xyz[1]; o[4] = (float)xyz[2]; o[5] = (float)xyz[0];
    }
    return n;
}

// transformLast after the latest update (LeGO transform order)
int slo_pg_last_transform(slo_pg* g, float out[6]) {
    if (!g || !out) return SLO_E_ARG;
    for (int k = 0; k < 6; ++k) out[k] = (float)g->last[k];
    return SLO_OK;
}

}  // extern "C"
