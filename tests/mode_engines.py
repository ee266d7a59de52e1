"""The oracle engine of Mode S (test infrastructure): the CPU restatement's
OracleStream.front / back / odom / mapstage (oracle/oracle_api.cpp) behind
the engine interface of slo_amd.modes' rank drivers, so the gloo rehearsal
(tests/test_modes_gloo.py) runs the same run_rank / run_rank3 as the GPU
ranks.  A scan is the numpy point array itself; buffers are numpy uint8
arrays (the transport allocates on receive)."""
import oracle_py as O


class OracleEngine:
    def __init__(self, cfg, fronts=1, split_back=False):
        self.fronts = [O.OracleStream(cfg) for _ in range(fronts)]
        self.owner = O.OracleStream(cfg)
        # split_back: odometry on self.odo, mapping on self.owner (OracleStream.odom / mapstage)
        self.odo = O.OracleStream(cfg) if split_back else None

    # ---- the one-process form (scan = points)
    def front(self, slot, pts, t, carry):
        return self.fronts[slot].front(pts, t, carry)

    def back(self, features, pts, t):
        if self.odo is not None:
            return self.mapping(self.odometry(features, t), pts, t)
        return self.owner.back(features, pts, t)

    def odometry(self, features, t):
        return self.odo.odom(features, t)

    def mapping(self, odom, pts, t):
        return self.owner.mapstage(odom, pts, t)

    # ---- the rank interface of slo_amd.modes.run_rank / run_rank3
    def recv_buffer(self, tag):
        return None

    def rank_front(self, scan, t, carry_in, need_carry):
        return self.front(0, scan, t, carry_in)

    def rank_back(self, features, scan, t):
        return self.back(features, scan, t)

    def rank_odometry(self, features, scan, t):
        return self.odometry(features, t)

    def rank_mapping(self, odom, scan, t):
        return self.mapping(odom, scan, t)
