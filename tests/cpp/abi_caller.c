/* A plain C99 translation unit against the public header alone
 * (include/slo_abi.h + include/slo_config.h), linked to libslo.so — the way a
 * ROS node or any FFI would bind the drop-in boundary.  Runs without a GPU:
 * presets, argument checks, the record layout, the host generator and the
 * host-side pose graph.  Prints "abi_caller ok" and exits 0 on success. */
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include "slo_abi.h"

#define CHECK(c) do { if (!(c)) { fprintf(stderr, "FAILED %s:%d: %s\n", __FILE__, __LINE__, #c); return 1; } } while (0)

int main(void) {
    slo_config cfg;
    CHECK(slo_config_preset(SLO_PRESET_HDL64_1800, &cfg) == SLO_OK);
    CHECK(cfg.n_scan == 64 && cfg.horizon_scan == 1800 && cfg.sc_num_ring == 20 && cfg.sc_num_sector == 60);
    CHECK(cfg.loop_closure_enable == 1 && cfg.pose_graph == 0);
    CHECK(slo_config_preset(99, &cfg) != SLO_OK);

    /* argument errors come back as codes, not crashes */
    slo_ctx* ctx = NULL;
    CHECK(slo_create(NULL, 0, 1, &ctx) == SLO_E_ARG);
    CHECK(slo_batch_process(NULL, NULL, NULL, 0.0) == SLO_E_ARG);
    CHECK(slo_graph_mode(NULL, 1) == SLO_E_ARG);
    CHECK(slo_pipeline(NULL, 6) == SLO_E_ARG);
    CHECK(slo_prepare_mapping(NULL) == SLO_E_ARG);
    CHECK(slo_record_floats() == SLO_RECORD_FLOATS);
    /* argument checks of the SCManager helpers and the batched VoxelGrid (no GPU call) */
    {
        double d[1200] = {0}, k[60] = {0}, dist = 0;
        int32_t sh = 0;
        CHECK(slo_sc_make_scancontext(NULL, NULL, 0, 16, 0, d) == SLO_E_ARG);
        CHECK(slo_sc_ring_key(NULL, d, k) == SLO_E_ARG);
        CHECK(slo_sc_sector_key(NULL, d, k) == SLO_E_ARG);
        CHECK(slo_sc_fast_align(NULL, k, k, &sh) == SLO_E_ARG);
        CHECK(slo_sc_dist_direct(NULL, d, d, &dist) == SLO_E_ARG);
        CHECK(slo_sc_distance(NULL, d, d, &dist, &sh) == SLO_E_ARG);
        CHECK(slo_batch_sc_distance(NULL, d, d, 1, &dist, &sh) == SLO_E_ARG);
        CHECK(slo_batch_voxel_grid(NULL, d, 1, NULL, 0.5f, d, 1, NULL, 1) == SLO_E_ARG);
        CHECK(slo_front_process(NULL, d, NULL, 0.0, NULL, d, d) == SLO_E_ARG);
        CHECK(slo_front_process(NULL, d, NULL, 0.0, NULL, NULL, NULL) == SLO_E_ARG);
        CHECK(slo_back_process(NULL, d, d, NULL, 0.0) == SLO_E_ARG);
        CHECK(slo_modes_carry_bytes(NULL) == 0 && slo_modes_features_bytes(NULL) == 0);
        CHECK(slo_odom_process(NULL, d, d, NULL, 0.0, d) == SLO_E_ARG);
        CHECK(slo_map_process(NULL, d, d, NULL, 0.0) == SLO_E_ARG);
        CHECK(slo_modes_odom_bytes(NULL) == 0);
        CHECK(cfg.voxel_order == SLO_VOXEL_PCL);
    }
    CHECK(SLO_REC_DESC + 20 * 60 <= SLO_RECORD_FLOATS);

    /* the synthetic stream generator (host) */
    CHECK(slo_config_preset(SLO_PRESET_VLP16, &cfg) == SLO_OK);
    float* pts = (float*)malloc(sizeof(float) * 4 * (size_t)cfg.max_points);
    CHECK(pts != NULL);
    int n = slo_gen_scan(SLO_PRESET_VLP16, 1, 0, 3, pts);
    CHECK(n == cfg.max_points);
    int finite = 0;
    for (int i = 0; i < n; ++i) finite += isfinite(pts[4 * i]) ? 1 : 0;
    CHECK(finite > n / 2 && finite < n);
    free(pts);

    /* the pose graph (host code): a three-pose chain with a consistent loop */
    slo_pg* g = NULL;
    CHECK(slo_pg_create(&g) == SLO_OK);
    float t[6] = {0, 0, 0, 0, 0, 0}, out[6], key[6];
    for (int k = 0; k < 3; ++k) {
        t[5] = (float)k;   /* 1 m steps along the camera-frame z (lidar x) */
        CHECK(slo_pg_add_keyframe(g, t, out, key) == SLO_OK);
    }
    CHECK(slo_pg_size(g) == 3);
    const float from[6] = {0, 0, 0, 0, 0, 0}, to[6] = {0, 0, 0, -2, 0, 0};
    CHECK(slo_pg_add_loop(g, 2, 0, from, to) == SLO_OK);
    int iters = 0;
    double cost = -1;
    CHECK(slo_pg_optimize(g, 0, &iters, &cost) == SLO_OK);
    CHECK(cost >= 0 && cost < 1e-9);
    float poses[18];
    CHECK(slo_pg_get_key_poses(g, poses, 3) == 3);
    CHECK(fabsf(poses[6 * 2 + 2] - 2.0f) < 1e-5f);   /* cloudKeyPoses6D z = camera z */
    CHECK(slo_pg_add_loop(g, 0, 7, from, to) == SLO_E_ARG);
    slo_pg_destroy(g);
    printf("abi_caller ok\n");
    return 0;
}
