"""Independent numpy model of LocalInertialBA's graph (optimizer.cc:2461-2781)
for pinning the oracle: edge errors only, Jacobians by central differences
through the reference's vertex updates (ImuCamPose::Update on VertexPose,
additive VertexVelocity / GyroBias / AccBias / VertexSBAPointXYZ), Huber
weights, the full (key frames + points) Gauss-Newton system, and one LM step
as a dense solve of (H + lambda I) x = b."""
from __future__ import annotations

import numpy as np

from inertial_cases import G, exp_so3, log_so3, polar

D_MONO = float(np.float32(np.sqrt(5.991)))
D_STEREO = float(np.float32(np.sqrt(7.815)))
D_IMU = float(np.sqrt(16.92))


def state21(s) -> np.ndarray:
    return np.concatenate([s["Rwb"].astype(float), s["twb"].astype(float), s["v"].astype(float),
                           s["bg"].astype(float), s["ba"].astype(float)])


def cam_of(c, x21, init=None):
    """Rcw, tcw of a key frame state: the ImuCamPose's camera pose (the
    initial estimate keeps the float pose the constructor read)."""
    if init is not None:
        return init["Rcw"].astype(float).reshape(3, 3), init["tcw"].astype(float)
    R, t = x21[:9].reshape(3, 3), x21[9:12]
    Rcb = c["Rcb"].astype(float).reshape(3, 3)
    return Rcb @ R.T, Rcb @ (-R.T @ t) + c["tcb"].astype(float)


def vis_error(c, Rcw, tcw, X, e):
    Xc = Rcw @ X + tcw
    u = float(c["fx"]) * Xc[0] / Xc[2] + float(c["cx"])
    v = float(c["fy"]) * Xc[1] / Xc[2] + float(c["cy"])
    if e["ur"] >= 0:
        return np.array([e["u"] - u, e["v"] - v, e["ur"] - (u - float(c["bf"]) / Xc[2])])
    return np.array([e["u"] - u, e["v"] - v])


def imu_errors(ie, x1, x2):
    """[(error, Omega, huber delta or None)] of EdgeInertial, EdgeGyroRW, EdgeAccRW."""
    pi = ie["preint"]
    dt = float(pi["dT"])
    R1, t1, v1, bg1, ba1 = x1[:9].reshape(3, 3), x1[9:12], x1[12:15], x1[15:18], x1[18:21]
    R2, t2, v2, bg2, ba2 = x2[:9].reshape(3, 3), x2[9:12], x2[12:15], x2[15:18], x2[18:21]
    dbg = bg1.astype(np.float32).astype(float) - pi["bg"].astype(float)
    dba = ba1.astype(np.float32).astype(float) - pi["ba"].astype(float)
    JRg, JVg, JVa, JPg, JPa = (pi[k].astype(float).reshape(3, 3) for k in
                               ("JRg", "JVg", "JVa", "JPg", "JPa"))
    dR = polar(pi["dR"].astype(float).reshape(3, 3) @ exp_so3(JRg @ dbg))
    dV = pi["dV"].astype(float) + JVg @ dbg + JVa @ dba
    dP = pi["dP"].astype(float) + JPg @ dbg + JPa @ dba
    er = log_so3(dR.T @ R1.T @ R2)
    ev = R1.T @ (v2 - v1 - G * dt) - dV
    ep = R1.T @ (t2 - t1 - v1 * dt - G * dt * dt / 2) - dP
    info = pi["info"].reshape(9, 9) * (1e-2 if ie["flags"] & 2 else 1.0)
    return [(np.r_[er, ev, ep], info, D_IMU if ie["flags"] & 1 else None),
            (bg2 - bg1, pi["info_g"].reshape(3, 3), None),
            (ba2 - ba1, pi["info_a"].reshape(3, 3), None)]


def update21(x, d, blk):
    R, t, v, bg, ba = (x[:9].reshape(3, 3).copy(), x[9:12].copy(), x[12:15].copy(),
                       x[15:18].copy(), x[18:21].copy())
    if blk == "P":
        t = t + R @ d[3:6]
        R = R @ exp_so3(d[:3])
    elif blk == "V":
        v = v + d
    elif blk == "G":
        bg = bg + d
    else:
        ba = ba + d
    return np.concatenate([R.ravel(), t, v, bg, ba])


def huber_w(e2, delta):
    return 1.0 if e2 <= delta * delta else delta / np.sqrt(e2)


def huber_rho(e2, delta):
    return e2 if e2 <= delta * delta else 2 * delta * np.sqrt(e2) - delta * delta


class Window:
    """The problem's states as the numpy model sees them."""

    def __init__(self, pb):
        self.pb = pb
        self.x = [state21(s) for s in pb.kfs]
        self.init = [s for s in pb.kfs]  # camera pose of a not-yet-updated vertex
        self.X = [p.astype(float) for p in pb.pts_init]
        self.free = [k for k in range(len(pb.kfs)) if not pb.fixed[k]]
        # a key frame's vertices: VP VV VG VA, or VP alone without IMU data
        # (optimizer.cc:2466-2484)
        self.blocks = {k: (("P", 0, 6), ("V", 6, 3), ("G", 9, 3), ("A", 12, 3)) if pb.imu[k] else (("P", 0, 6),)
                       for k in self.free}
        self.col, o = {}, 0
        for k in self.free:
            self.col[k] = o
            o += 15 if pb.imu[k] else 6
        self.n_kf_rows = o
        self.n = o + 3 * len(self.X)

    def errors(self, x=None, X=None, init=None):
        """[(error, Omega, delta)] visual edges in order, then per IMU link its three edges."""
        pb, c = self.pb, self.pb.calib
        x = self.x if x is None else x
        X = self.X if X is None else X
        init = self.init if init is None else init
        out = []
        for e in pb.edges:
            Rcw, tcw = cam_of(c, x[e["kf"]], init[e["kf"]])
            err = vis_error(c, Rcw, tcw, X[e["point"]], e)
            out.append((err, np.eye(len(err)) * float(e["inv_sigma2"]),
                        D_STEREO if e["ur"] >= 0 else D_MONO))
        for ie in pb.imu_edges:
            out += imu_errors(ie, x[ie["kf1"]], x[ie["kf2"]])
        return out

    def robust_chi2(self):
        return sum(huber_rho(float(e @ Om @ e), d) if d is not None else float(e @ Om @ e)
                   for e, Om, d in self.errors())

    def system(self, h=1e-6):
        base = self.errors()
        Js = [np.zeros((len(e), self.n)) for e, _, _ in base]
        for k in self.free:
            for blk, off, dim in self.blocks[k]:
                for j in range(dim):
                    d = np.zeros(dim)
                    d[j] = h
                    res = []
                    for sg in (1, -1):
                        x = list(self.x)
                        x[k] = update21(self.x[k], sg * d, blk)
                        init = list(self.init)
                        if blk == "P":
                            init[k] = None  # the update rebuilds Rcw / tcw
                        res.append(self.errors(x=x, init=init))
                    for i, (ep, em) in enumerate(zip(*res)):
                        Js[i][:, self.col[k] + off + j] = (ep[0] - em[0]) / (2 * h)
        o0 = self.n_kf_rows
        for p in range(len(self.X)):
            for j in range(3):
                res = []
                for sg in (1, -1):
                    X = list(self.X)
                    X[p] = self.X[p] + sg * h * np.eye(3)[j]
                    res.append(self.errors(X=X))
                for i, (ep, em) in enumerate(zip(*res)):
                    Js[i][:, o0 + 3 * p + j] = (ep[0] - em[0]) / (2 * h)
        H = np.zeros((self.n, self.n))
        b = np.zeros(self.n)
        for (e, Om, d), J in zip(base, Js):
            w = huber_w(float(e @ Om @ e), d) if d is not None else 1.0
            H += J.T @ (w * Om) @ J
            b -= J.T @ (w * Om) @ e
        return H, b

    def step(self, lam, system=None):
        """One LM trial: (H + lam I) x = b (by default the numeric system),
        the vertex updates applied."""
        H, b = self.system() if system is None else system
        dx = np.linalg.solve(H + lam * np.eye(self.n), b)
        x = list(self.x)
        for k in self.free:
            o = self.col[k]
            xk = self.x[k]
            for blk, off, dim in self.blocks[k]:
                xk = update21(xk, dx[o + off:o + off + dim], blk)
            x[k] = xk
        o0 = self.n_kf_rows
        X = [self.X[p] + dx[o0 + 3 * p:o0 + 3 * p + 3] for p in range(len(self.X))]
        return x, X
