// nanoflann_pin.cpp — TEST INFRASTRUCTURE ONLY (fixture generator).
//
// Runs the reference's own ring-key tree — KDTreeVectorOfVectorsAdaptor<
// std::vector<std::vector<float>>, float> with max leaf 10 over the snapshot,
// KNNResultSet<float> into zero-initialised index/distance vectors,
// findNeighbors(..., SearchParams(10)) — exactly as Scancontext.cpp:270-289
// calls it.  Compiled by `make -C oracle ref` against the vendored headers in
// /root/reference/SC-LeGO-LOAM/LeGO-LOAM/include (nothing is copied; the
// binary goes to oracle/_ref/ and is only run by tests/golden/make_golden.py).
//
// stdin  (binary): int32 dim, int32 K, int32 n_queries, then per query:
//                  int32 n_snapshot, float snapshot[n_snapshot][dim], float q[dim]
// stdout (binary): per query uint64 idx[K], float dist[K]
#include <KDTreeVectorOfVectorsAdaptor.h>

#include <cstdint>
#include <cstdio>
#include <memory>
#include <vector>

using KeyMat = std::vector<std::vector<float>>;
using InvKeyTree = KDTreeVectorOfVectorsAdaptor<KeyMat, float>;

static bool rd(void* p, size_t n) { return fread(p, 1, n, stdin) == n; }

int main() {
    int32_t dim, K, nq;
    if (!rd(&dim, 4) || !rd(&K, 4) || !rd(&nq, 4)) return 1;
    for (int q = 0; q < nq; ++q) {
        int32_t n;
        if (!rd(&n, 4) || n <= 0) return 2;
        KeyMat snap(n, std::vector<float>(dim));
        for (auto& row : snap)
            if (!rd(row.data(), sizeof(float) * dim)) return 3;
        std::vector<float> key(dim);
        if (!rd(key.data(), sizeof(float) * dim)) return 4;
        std::unique_ptr<InvKeyTree> tree = std::make_unique<InvKeyTree>(dim, snap, 10);
        std::vector<size_t> idx(K);
        std::vector<float> dist(K);
        nanoflann::KNNResultSet<float> rs(K);
        rs.init(&idx[0], &dist[0]);
        tree->index->findNeighbors(rs, &key[0], nanoflann::SearchParams(10));
        for (int k = 0; k < K; ++k) {
            uint64_t v = idx[k];
            fwrite(&v, 8, 1, stdout);
        }
        fwrite(dist.data(), sizeof(float), K, stdout);
    }
    return 0;
}
