"""CPU restatement of mapOptimization's pose graph — TEST INFRASTRUCTURE ONLY.

Only tests/ may import this; the product path is csrc/slo_pg.hip.  It states
the factor graph the reference hands GTSAM iSAM2 (SC-LeGO-LOAM
LeGO-LOAM/src/mapOptmization.cpp):
  prior on key pose 0, variances (1e-6,1e-6,1e-6,1e-8,1e-8,1e-6)   MO:365-368, 1541-1546
  odometry BetweenFactor(k-1, k, transformLast.between(transformAftMapped))  MO:1547-1555
  loop BetweenFactor(from, to, poseFrom.between(poseTo)), Cauchy(1) on
  variances 0.5                                                     MO:985-997, 1038-1046, 1083-1091
  correctPoses → cloudKeyPoses6D                                    MO:1642-1664
and solves it densely (numpy) by iteratively re-weighted Gauss-Newton with a
step-halving line search.  SO(3) exp/log come from scipy's Rotation, not the
product's formulas.

PARITY UNPINNED against GTSAM itself: GTSAM is not in this image and the
reference holds no pose-graph fixtures, so this restatement checks the
product's solver on the same factor graph (GTSAM 4 expmap conventions:
tangent [rot, trans], retract T*Exp(d), between error Log(Z^-1 Ti^-1 Tj)).
"""
import numpy as np
from scipy.spatial.transform import Rotation

ODO_VAR = np.array([1e-6, 1e-6, 1e-6, 1e-8, 1e-8, 1e-6])
LOOP_VAR = 0.5


def rzryrx(x, y, z):
    return Rotation.from_euler("ZYX", [z, y, x]).as_matrix()     # Rz(z) Ry(y) Rx(x)


def pose(x, y, z, tx, ty, tz):
    T = np.eye(4)
    T[:3, :3] = rzryrx(x, y, z)
    T[:3, 3] = [tx, ty, tz]
    return T


def from_transform(t):        # Pose3(RzRyRx(t2, t0, t1), Point3(t5, t3, t4))
    t = np.asarray(t, np.float64)
    return pose(t[2], t[0], t[1], t[5], t[3], t[4])


def xyz(R):
    z, y, x = Rotation.from_matrix(R).as_euler("ZYX")
    return np.array([x, y, z])


def to_key_pose6d(T):         # x=t.y y=t.z z=t.x roll=pitch() pitch=yaw() yaw=roll()
    r = xyz(T[:3, :3])
    return np.array([T[1, 3], T[2, 3], T[0, 3], r[1], r[2], r[0]])


def to_rzryrx_args(T):        # the Pose3(RzRyRx(v0,v1,v2), Point3(v3,v4,v5)) arguments
    return np.concatenate([xyz(T[:3, :3]), T[:3, 3]])


def _V(w):
    th = np.linalg.norm(w)
    W = np.array([[0, -w[2], w[1]], [w[2], 0, -w[0]], [-w[1], w[0], 0]])
    if th < 1e-8:
        return np.eye(3) + W / 2
    return np.eye(3) + (1 - np.cos(th)) / th**2 * W + (th - np.sin(th)) / th**3 * W @ W


def exp(d):
    T = np.eye(4)
    T[:3, :3] = Rotation.from_rotvec(d[:3]).as_matrix()
    T[:3, 3] = _V(d[:3]) @ d[3:]
    return T


def log(T):
    w = Rotation.from_matrix(T[:3, :3]).as_rotvec()
    return np.concatenate([w, np.linalg.solve(_V(w), T[:3, 3])])


class Graph:
    def __init__(self):
        self.est, self.fac, self.last = [], [], None

    def add_keyframe(self, transform):
        t = np.asarray(transform, np.float32).astype(np.float64)
        if not self.est:
            T = from_transform(t)
            self.fac.append((0, -1, np.linalg.inv(T), 1 / np.sqrt(ODO_VAR), False))
            self.est.append(T)
            self.last = t
            return
        z = np.linalg.inv(from_transform(self.last)) @ from_transform(t)
        n = len(self.est)
        self.fac.append((n - 1, n, np.linalg.inv(z), 1 / np.sqrt(ODO_VAR), False))
        self.est.append(self.est[-1] @ z)
        T = self.est[-1]
        r = xyz(T[:3, :3])
        self.last = np.array([r[1], r[2], r[0], T[1, 3], T[2, 3], T[0, 3]])

    def add_loop(self, i, j, pose_from, pose_to):
        a = pose(*np.asarray(pose_from, np.float32).astype(np.float64))
        b = pose(*np.asarray(pose_to, np.float32).astype(np.float64))
        self.fac.append((i, j, np.linalg.inv(np.linalg.inv(a) @ b), np.full(6, 1 / np.sqrt(LOOP_VAR)), True))

    def _err(self, f, x):
        i, j, Zi, s, _ = f
        h = x[i] if j < 0 else np.linalg.inv(x[i]) @ x[j]
        return log(Zi @ h) * s

    def cost(self, x):
        c = 0.0
        for f in self.fac:
            r2 = float(self._err(f, x) @ self._err(f, x))
            c += 0.5 * np.log1p(r2) if f[4] else 0.5 * r2
        return c

    def optimize(self, iters=50):
        n = len(self.est)
        for _ in range(iters):
            H = np.zeros((6 * n, 6 * n))
            g = np.zeros(6 * n)
            for f in self.fac:
                e = self._err(f, self.est)
                w = 1 / (1 + e @ e) if f[4] else 1.0
                blocks = [f[0]] if f[1] < 0 else [f[0], f[1]]
                J = {}
                for p in blocks:
                    Jp = np.zeros((6, 6))
                    for c in range(6):
                        d = np.zeros(6)
                        d[c] = 1e-6
                        xp = list(self.est); xp[p] = self.est[p] @ exp(d)
                        xm = list(self.est); xm[p] = self.est[p] @ exp(-d)
                        Jp[:, c] = (self._err(f, xp) - self._err(f, xm)) / 2e-6
                    J[p] = Jp
                for a in blocks:
                    g[6 * a:6 * a + 6] -= w * J[a].T @ e
                    for b in blocks:
                        H[6 * a:6 * a + 6, 6 * b:6 * b + 6] += w * J[a].T @ J[b]
            dx = np.linalg.solve(H, g)
            c0, step = self.cost(self.est), 1.0
            while step > 1e-4:
                trial = [self.est[p] @ exp(step * dx[6 * p:6 * p + 6]) for p in range(n)]
                if self.cost(trial) <= c0:
                    break
                step *= 0.5
            else:
                break
            self.est = trial
            if c0 - self.cost(trial) <= 1e-12 * max(c0, 1e-300):
                break
        return self.cost(self.est)

    def key_poses(self):
        return np.array([to_key_pose6d(T) for T in self.est])


class PipelineWithGraph:
    """TEST INFRASTRUCTURE: the oracle pipeline (oracle_py.OracleStream) with
    this numpy graph as its back end, driven in the order slo_pgwire.hip
    follows (mapOptmization.cpp): after each mapping step the saved keyframe
    adds its odometry factor and, once a loop is closed, the estimate is
    written back (saveKeyFramesAndFactor MO:1541-1611 + correctPoses
    MO:1642-1664); after SC detect + verification, accepted RS / SC
    candidates add Cauchy loop factors and the graph is solved
    (MO:1030-1046, 1078-1091)."""

    def __init__(self, stream, graph=None):
        self.st, self.g, self.pending, self.snap = stream, graph if graph is not None else Graph(), False, None
        self.loops = 0

    def step(self, pts, t):
        import oracle_py as O
        f = self.st.step_map(pts, t)
        if f & 2:
            if f & 4:
                self.g.add_keyframe(self.st.get("kf_pre"))
                if self.pending:
                    tf = self.g.last if len(self.g.est) > 1 else None
                    self.st.set_key_poses(self.g.key_poses().astype(np.float32),
                                          None if tf is None else np.asarray(tf, np.float32))
                    self.pending = False
            elif self.pending:
                self.st.set_key_poses(self.snap)
                self.pending = False
        f |= self.st.step_loop(f, t)
        if (f & 8) and (f & 4):
            lp = self.st.get("loop")
            if len(lp) == 2:
                rs, sc = lp[0], lp[1]
                use_rs = rs["ran"] and rs["accepted"] and rs["id"] >= 0
                use_sc = sc["ran"] and sc["accepted"] and sc["id"] >= 0
                latest = len(self.g.est) - 1
                # aLoopIsClosed = true once performLoopClosure got past
                # detection, accepted or not (MO:1107-1108)
                if (rs["ran"] or sc["ran"]) and latest >= 0:
                    self.snap = self.g.key_poses().astype(np.float32)
                    kp = self.st.get("keyposes").reshape(-1, 6)
                    if use_rs:
                        frm = O.rs_loop_from(rs["xyzrpy"], kp[latest])
                        p = kp[rs["id"]]
                        to = np.array([p[5], p[3], p[4], p[2], p[0], p[1]], np.float32)
                        self.g.add_loop(latest, int(rs["id"]), frm, to)
                    if use_sc:
                        x = np.asarray(sc["xyzrpy"], np.float32)
                        self.g.add_loop(latest, int(sc["id"]), np.array([x[3], x[4], x[5], x[0], x[1], x[2]], np.float32),
                                        np.zeros(6, np.float32))
                    if use_rs or use_sc:
                        self.g.optimize()
                        self.loops += 1
                    self.pending = True
        return f
