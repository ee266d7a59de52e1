// oracle_mo.h — TEST INFRASTRUCTURE ONLY: CPU restatement of the scan-to-map
// half of mapOptmization.cpp: transformAssociateToMap 397-482,
// transformUpdate 484-517 (no IMU), pointAssociateToMap 519-548,
// transformPointCloud 550-596, laserOdometryHandler 655-667,
// extractSurroundingKeyFrames 1122-1231 (loopClosureEnableFlag branch),
// downsampleCurrentScan 1233-1263, cornerOptimization 1265-1346,
// surfOptimization 1348-1399, LMOptimization 1401-1499,
// scan2MapOptimization 1501-1522, saveKeyFramesAndFactor 1525-1639 minus
// GTSAM.  With only a prior and consistent between-factors (no loop factor is
// ever added on this path) the iSAM2 estimate of the newest node is its
// initial value, so the keyframe pose is transformTobeMapped /
// transformAftMapped; the tf quaternion round trip (FA:1728 -> MO:659) and the
// Rot3 RzRyRx <-> rpy round trip are identities after float rounding except
// with probability ~2^-29 per value (DESIGN.md "pose-graph boundary").
#pragma once

#include "oracle_sc.h"
#include "oracle_tf.h"
#include <deque>

namespace oracle {

struct Pose6 { float x, y, z, roll, pitch, yaw; };

struct MapOptimization {
    slo_config cfg;
    bool stable_voxel = false;
    float transformLast[6] = {0}, transformSum[6] = {0}, transformIncre[6] = {0};
    float transformTobeMapped[6] = {0}, transformBefMapped[6] = {0}, transformAftMapped[6] = {0};
    std::vector<Cloud> cornerCloudKeyFrames, surfCloudKeyFrames, outlierCloudKeyFrames;
    std::vector<Pose6> keyPoses;  // cloudKeyPoses6D (3D = x,y,z)
    std::vector<double> keyTimes; // cloudKeyPoses6D[i].time (MO:1609: timeLaserOdometry)
    double timeLaserOdometry = 0;
    std::deque<Cloud> recentCorner, recentSurf, recentOutlier;
    int latestFrameID = 0;
    // loopClosureEnableFlag == false: the keyframes of the local map, in order (MO:1181-1214)
    std::vector<int> surroundingExistingKeyPosesID;
    std::vector<Cloud> surroundingCorner, surroundingSurf, surroundingOutlier;
    Pt previousRobotPosPoint{0, 0, 0, 0}, currentRobotPosPoint{0, 0, 0, 0};
    double timeLastProcessing = -1;
    Cloud laserCloudRaw, laserCloudRawDS, laserCloudCornerLast, laserCloudSurfLast, laserCloudOutlierLast;
    Cloud laserCloudCornerLastDS, laserCloudSurfLastDS, laserCloudOutlierLastDS;
    Cloud laserCloudSurfTotalLast, laserCloudSurfTotalLastDS;
    Cloud laserCloudCornerFromMap, laserCloudSurfFromMap, laserCloudCornerFromMapDS, laserCloudSurfFromMapDS;
    Cloud lastCornerMapDS, lastSurfMapDS;   // the last run's DS maps (parity checks only)
    Cloud lastCornerMapRaw, lastSurfMapRaw; // and the maps before their VoxelGrid (parity checks only)
    Cloud laserCloudOri, coeffSel;
    KdTree kdtreeCornerFromMap, kdtreeSurfFromMap;
    bool isDegenerate = false;
    float matP[36] = {0};
    float cRoll = 0, sRoll = 0, cPitch = 0, sPitch = 0, cYaw = 0, sYaw = 0, tX = 0, tY = 0, tZ = 0;
    SCManager sc;
    // per-run stats
    int lm_iters = 0;
    bool ran = false, saved_keyframe = false;
    // /aft_mapped_to_init as TransformFusion decodes it (publishTF MO:680-705 -> TF:222-241)
    float tfAft[6] = {0}, tfBef[6] = {0};
    // the transform the last saved keyframe hands to the pose graph (MO:1541-1555)
    float kfPre[6] = {0};

    // correctPoses (MO:1642-1664) from a pose-graph estimate: key poses
    // [0, n), the recent deques cleared; transform (may be null) becomes
    // transformAftMapped / Last / TobeMapped (MO:1601-1611) and publishTF
    // hands it on (MO:1701)
    void set_key_poses(const float* poses6, int n, const float* transform) {
        for (int i = 0; i < n && i < (int)keyPoses.size(); ++i)
            keyPoses[i] = Pose6{poses6[6 * i], poses6[6 * i + 1], poses6[6 * i + 2], poses6[6 * i + 3],
                                poses6[6 * i + 4], poses6[6 * i + 5]};
        if (transform) {
            for (int k = 0; k < 6; ++k) { transformAftMapped[k] = transform[k]; transformLast[k] = transform[k]; transformTobeMapped[k] = transform[k]; }
            odom_handoff(transformAftMapped, tfAft);
        }
        recentCorner.clear(); recentSurf.clear(); recentOutlier.clear();
    }

    explicit MapOptimization(const slo_config& c) : cfg(c), sc(c) {}

    // transformAssociateToMap (MO:397-482); TransformFusion (transformFusion.cpp:94-181)
    // evaluates the same expressions on its own copies of the three transforms
    static void associate_to_map(const float* transformSum, const float* transformBefMapped,
                                 const float* transformAftMapped, float* transformIncre,
                                 float* transformTobeMapped) {
        using namespace oracle_libm;
        float x1 = cosf_(transformSum[1]) * (transformBefMapped[3] - transformSum[3]) -
                   sinf_(transformSum[1]) * (transformBefMapped[5] - transformSum[5]);
        float y1 = transformBefMapped[4] - transformSum[4];
        float z1 = sinf_(transformSum[1]) * (transformBefMapped[3] - transformSum[3]) +
                   cosf_(transformSum[1]) * (transformBefMapped[5] - transformSum[5]);
        float x2 = x1;
        float y2 = cosf_(transformSum[0]) * y1 + sinf_(transformSum[0]) * z1;
        float z2 = -sinf_(transformSum[0]) * y1 + cosf_(transformSum[0]) * z1;
        transformIncre[3] = cosf_(transformSum[2]) * x2 + sinf_(transformSum[2]) * y2;
        transformIncre[4] = -sinf_(transformSum[2]) * x2 + cosf_(transformSum[2]) * y2;
        transformIncre[5] = z2;
        float sbcx = sinf_(transformSum[0]), cbcx = cosf_(transformSum[0]);
        float sbcy = sinf_(transformSum[1]), cbcy = cosf_(transformSum[1]);
        float sbcz = sinf_(transformSum[2]), cbcz = cosf_(transformSum[2]);
        float sblx = sinf_(transformBefMapped[0]), cblx = cosf_(transformBefMapped[0]);
        float sbly = sinf_(transformBefMapped[1]), cbly = cosf_(transformBefMapped[1]);
        float sblz = sinf_(transformBefMapped[2]), cblz = cosf_(transformBefMapped[2]);
        float salx = sinf_(transformAftMapped[0]), calx = cosf_(transformAftMapped[0]);
        float saly = sinf_(transformAftMapped[1]), caly = cosf_(transformAftMapped[1]);
        float salz = sinf_(transformAftMapped[2]), calz = cosf_(transformAftMapped[2]);
        float srx = -sbcx * (salx * sblx + calx * cblx * salz * sblz + calx * calz * cblx * cblz) -
                    cbcx * sbcy * (calx * calz * (cbly * sblz - cblz * sblx * sbly) -
                                   calx * salz * (cbly * cblz + sblx * sbly * sblz) + cblx * salx * sbly) -
                    cbcx * cbcy * (calx * salz * (cblz * sbly - cbly * sblx * sblz) -
                                   calx * calz * (sbly * sblz + cbly * cblz * sblx) + cblx * cbly * salx);
        transformTobeMapped[0] = -asinf_(srx);
        float srycrx = sbcx * (cblx * cblz * (caly * salz - calz * salx * saly) -
                               cblx * sblz * (caly * calz + salx * saly * salz) + calx * saly * sblx) -
                       cbcx * cbcy * ((caly * calz + salx * saly * salz) * (cblz * sbly - cbly * sblx * sblz) +
                                      (caly * salz - calz * salx * saly) * (sbly * sblz + cbly * cblz * sblx) -
                                      calx * cblx * cbly * saly) +
                       cbcx * sbcy * ((caly * calz + salx * saly * salz) * (cbly * cblz + sblx * sbly * sblz) +
                                      (caly * salz - calz * salx * saly) * (cbly * sblz - cblz * sblx * sbly) +
                                      calx * cblx * saly * sbly);
        float crycrx = sbcx * (cblx * sblz * (calz * saly - caly * salx * salz) -
                               cblx * cblz * (saly * salz + caly * calz * salx) + calx * caly * sblx) +
                       cbcx * cbcy * ((saly * salz + caly * calz * salx) * (sbly * sblz + cbly * cblz * sblx) +
                                      (calz * saly - caly * salx * salz) * (cblz * sbly - cbly * sblx * sblz) +
                                      calx * caly * cblx * cbly) -
                       cbcx * sbcy * ((saly * salz + caly * calz * salx) * (cbly * sblz - cblz * sblx * sbly) +
                                      (calz * saly - caly * salx * salz) * (cbly * cblz + sblx * sbly * sblz) -
                                      calx * caly * cblx * sbly);
        transformTobeMapped[1] = atan2f_(srycrx / cosf_(transformTobeMapped[0]), crycrx / cosf_(transformTobeMapped[0]));
        float srzcrx = (cbcz * sbcy - cbcy * sbcx * sbcz) * (calx * salz * (cblz * sbly - cbly * sblx * sblz) -
                                                          calx * calz * (sbly * sblz + cbly * cblz * sblx) +
                                                          cblx * cbly * salx) -
                       (cbcy * cbcz + sbcx * sbcy * sbcz) * (calx * calz * (cbly * sblz - cblz * sblx * sbly) -
                                                          calx * salz * (cbly * cblz + sblx * sbly * sblz) +
                                                          cblx * salx * sbly) +
                       cbcx * sbcz * (salx * sblx + calx * cblx * salz * sblz + calx * calz * cblx * cblz);
        float crzcrx = (cbcy * sbcz - cbcz * sbcx * sbcy) * (calx * calz * (cbly * sblz - cblz * sblx * sbly) -
                                                          calx * salz * (cbly * cblz + sblx * sbly * sblz) +
                                                          cblx * salx * sbly) -
                       (sbcy * sbcz + cbcy * cbcz * sbcx) * (calx * salz * (cblz * sbly - cbly * sblx * sblz) -
                                                          calx * calz * (sbly * sblz + cbly * cblz * sblx) +
                                                          cblx * cbly * salx) +
                       cbcx * cbcz * (salx * sblx + calx * cblx * salz * sblz + calx * calz * cblx * cblz);
        transformTobeMapped[2] = atan2f_(srzcrx / cosf_(transformTobeMapped[0]), crzcrx / cosf_(transformTobeMapped[0]));
        x1 = cosf_(transformTobeMapped[2]) * transformIncre[3] - sinf_(transformTobeMapped[2]) * transformIncre[4];
        y1 = sinf_(transformTobeMapped[2]) * transformIncre[3] + cosf_(transformTobeMapped[2]) * transformIncre[4];
        z1 = transformIncre[5];
        x2 = x1;
        y2 = cosf_(transformTobeMapped[0]) * y1 - sinf_(transformTobeMapped[0]) * z1;
        z2 = sinf_(transformTobeMapped[0]) * y1 + cosf_(transformTobeMapped[0]) * z1;
        transformTobeMapped[3] = transformAftMapped[3] - (cosf_(transformTobeMapped[1]) * x2 + sinf_(transformTobeMapped[1]) * z2);
        transformTobeMapped[4] = transformAftMapped[4] - y2;
        transformTobeMapped[5] = transformAftMapped[5] - (-sinf_(transformTobeMapped[1]) * x2 + cosf_(transformTobeMapped[1]) * z2);
    }

    void transformAssociateToMap() {
        associate_to_map(transformSum, transformBefMapped, transformAftMapped, transformIncre, transformTobeMapped);
    }

    void transformUpdate() {
        for (int i = 0; i < 6; i++) {
            transformBefMapped[i] = transformSum[i];
            transformAftMapped[i] = transformTobeMapped[i];
        }
    }

    void updatePointAssociateToMapSinCos() {
        using namespace oracle_libm;
        cRoll = cosf_(transformTobeMapped[0]); sRoll = sinf_(transformTobeMapped[0]);
        cPitch = cosf_(transformTobeMapped[1]); sPitch = sinf_(transformTobeMapped[1]);
        cYaw = cosf_(transformTobeMapped[2]); sYaw = sinf_(transformTobeMapped[2]);
        tX = transformTobeMapped[3]; tY = transformTobeMapped[4]; tZ = transformTobeMapped[5];
    }
    Pt pointAssociateToMap(const Pt& pi) const {
        float x1 = cYaw * pi.x - sYaw * pi.y;
        float y1 = sYaw * pi.x + cYaw * pi.y;
        float z1 = pi.z;
        float x2 = x1;
        float y2 = cRoll * y1 - sRoll * z1;
        float z2 = sRoll * y1 + cRoll * z1;
        return {cPitch * x2 + sPitch * z2 + tX, y2 + tY, -sPitch * x2 + cPitch * z2 + tZ, pi.intensity};
    }
    static Cloud transformPointCloud(const Cloud& in, const Pose6& t) {
        using namespace oracle_libm;
        float ctRoll = cosf_(t.roll), stRoll = sinf_(t.roll);
        float ctPitch = cosf_(t.pitch), stPitch = sinf_(t.pitch);
        float ctYaw = cosf_(t.yaw), stYaw = sinf_(t.yaw);
        Cloud out(in.size());
        for (size_t i = 0; i < in.size(); ++i) {
            const Pt& p = in[i];
            float x1 = ctYaw * p.x - stYaw * p.y;
            float y1 = stYaw * p.x + ctYaw * p.y;
            float z1 = p.z;
            float x2 = x1;
            float y2 = ctRoll * y1 - stRoll * z1;
            float z2 = stRoll * y1 + ctRoll * z1;
            out[i] = {ctPitch * x2 + stPitch * z2 + t.x, y2 + t.y, -stPitch * x2 + ctPitch * z2 + t.z, p.intensity};
        }
        return out;
    }

    // loopClosureEnableFlag == false (MO:1167-1222): radius search of the key
    // positions around currentRobotPosPoint (PCL KdTreeFLANN::radiusSearch:
    // FLANN L2 of query - point, kept when < (float)(radius * radius)), the
    // hits VoxelGrid'ed at leaf 1.0 with intensity = key index (so a voxel's
    // id is (int) of the mean of its members' indices, MO:1176-1183), then
    // the existing list updated in place: ids no longer present erased in
    // order, new ids appended in voxel order, their clouds transformed
    void extractSurroundingRadius() {
        const float r2 = (float)((double)cfg.surrounding_keyframe_search_radius *
                                 (double)cfg.surrounding_keyframe_search_radius);
        Cloud near;
        for (size_t i = 0; i < keyPoses.size(); ++i) {
            const Pt p{keyPoses[i].x, keyPoses[i].y, keyPoses[i].z, (float)i};
            if (sqdist(currentRobotPosPoint, p) < r2) near.push_back(p);
        }
        Cloud ds;
        voxel_grid(near, cfg.leaf_surrounding_key_poses, ds, stable_voxel);
        for (size_t i = 0; i < surroundingExistingKeyPosesID.size(); ++i) {
            bool existing = false;
            for (const Pt& q : ds)
                if (surroundingExistingKeyPosesID[i] == (int)q.intensity) { existing = true; break; }
            if (!existing) {
                surroundingExistingKeyPosesID.erase(surroundingExistingKeyPosesID.begin() + i);
                surroundingCorner.erase(surroundingCorner.begin() + i);
                surroundingSurf.erase(surroundingSurf.begin() + i);
                surroundingOutlier.erase(surroundingOutlier.begin() + i);
                --i;
            }
        }
        for (const Pt& q : ds) {
            const int k = (int)q.intensity;
            bool existing = false;
            for (int id : surroundingExistingKeyPosesID)
                if (id == k) { existing = true; break; }
            if (existing) continue;
            surroundingExistingKeyPosesID.push_back(k);
            surroundingCorner.push_back(transformPointCloud(cornerCloudKeyFrames[k], keyPoses[k]));
            surroundingSurf.push_back(transformPointCloud(surfCloudKeyFrames[k], keyPoses[k]));
            surroundingOutlier.push_back(transformPointCloud(outlierCloudKeyFrames[k], keyPoses[k]));
        }
        for (size_t i = 0; i < surroundingExistingKeyPosesID.size(); ++i) {
            laserCloudCornerFromMap.insert(laserCloudCornerFromMap.end(), surroundingCorner[i].begin(), surroundingCorner[i].end());
            laserCloudSurfFromMap.insert(laserCloudSurfFromMap.end(), surroundingSurf[i].begin(), surroundingSurf[i].end());
            laserCloudSurfFromMap.insert(laserCloudSurfFromMap.end(), surroundingOutlier[i].begin(), surroundingOutlier[i].end());
        }
    }

    void extractSurroundingKeyFrames() {
        if (keyPoses.empty()) return;
        if (!cfg.loop_closure_enable) {
            extractSurroundingRadius();
            voxel_grid(laserCloudCornerFromMap, cfg.leaf_corner, laserCloudCornerFromMapDS, stable_voxel);
            voxel_grid(laserCloudSurfFromMap, cfg.leaf_surf, laserCloudSurfFromMapDS, stable_voxel);
            return;
        }
        const int N = cfg.surrounding_keyframe_search_num;
        if ((int)recentCorner.size() < N) {
            recentCorner.clear(); recentSurf.clear(); recentOutlier.clear();
            int numPoses = (int)keyPoses.size();
            for (int i = numPoses - 1; i >= 0; --i) {
                int k = i;  // (int)cloudKeyPoses3D[i].intensity == i
                recentCorner.push_front(transformPointCloud(cornerCloudKeyFrames[k], keyPoses[k]));
                recentSurf.push_front(transformPointCloud(surfCloudKeyFrames[k], keyPoses[k]));
                recentOutlier.push_front(transformPointCloud(outlierCloudKeyFrames[k], keyPoses[k]));
                if ((int)recentCorner.size() >= N) break;
            }
        } else {
            if (latestFrameID != (int)keyPoses.size() - 1) {
                recentCorner.pop_front(); recentSurf.pop_front(); recentOutlier.pop_front();
                latestFrameID = (int)keyPoses.size() - 1;
                const Pose6& t = keyPoses[latestFrameID];
                recentCorner.push_back(transformPointCloud(cornerCloudKeyFrames[latestFrameID], t));
                recentSurf.push_back(transformPointCloud(surfCloudKeyFrames[latestFrameID], t));
                recentOutlier.push_back(transformPointCloud(outlierCloudKeyFrames[latestFrameID], t));
            }
        }
        for (size_t i = 0; i < recentCorner.size(); ++i) {
            laserCloudCornerFromMap.insert(laserCloudCornerFromMap.end(), recentCorner[i].begin(), recentCorner[i].end());
            laserCloudSurfFromMap.insert(laserCloudSurfFromMap.end(), recentSurf[i].begin(), recentSurf[i].end());
            laserCloudSurfFromMap.insert(laserCloudSurfFromMap.end(), recentOutlier[i].begin(), recentOutlier[i].end());
        }
        voxel_grid(laserCloudCornerFromMap, cfg.leaf_corner, laserCloudCornerFromMapDS, stable_voxel);
        voxel_grid(laserCloudSurfFromMap, cfg.leaf_surf, laserCloudSurfFromMapDS, stable_voxel);
    }

    void downsampleCurrentScan() {
        voxel_grid(laserCloudRaw, cfg.leaf_sc, laserCloudRawDS, stable_voxel);
        voxel_grid(laserCloudCornerLast, cfg.leaf_corner, laserCloudCornerLastDS, stable_voxel);
        voxel_grid(laserCloudSurfLast, cfg.leaf_surf, laserCloudSurfLastDS, stable_voxel);
        voxel_grid(laserCloudOutlierLast, cfg.leaf_outlier, laserCloudOutlierLastDS, stable_voxel);
        laserCloudSurfTotalLast.clear();
        laserCloudSurfTotalLast.insert(laserCloudSurfTotalLast.end(), laserCloudSurfLastDS.begin(), laserCloudSurfLastDS.end());
        laserCloudSurfTotalLast.insert(laserCloudSurfTotalLast.end(), laserCloudOutlierLastDS.begin(), laserCloudOutlierLastDS.end());
        voxel_grid(laserCloudSurfTotalLast, cfg.leaf_surf, laserCloudSurfTotalLastDS, stable_voxel);
    }

    void cornerOptimization(int) {
        updatePointAssociateToMapSinCos();
        int ind[5]; float dis[5];
        const int mapN = (int)laserCloudCornerFromMapDS.size();
        for (size_t i = 0; i < laserCloudCornerLastDS.size(); i++) {
            const Pt& pointOri = laserCloudCornerLastDS[i];
            Pt pointSel = pointAssociateToMap(pointOri);
            int cnt = kdtreeCornerFromMap.knn(pointSel, 5, ind, dis);
            if (cnt < 5 || mapN < 5) continue;
            if (dis[4] < 1.0) {
                const Cloud& M = laserCloudCornerFromMapDS;
                float cx = 0, cy = 0, cz = 0;
                for (int j = 0; j < 5; j++) { cx += M[ind[j]].x; cy += M[ind[j]].y; cz += M[ind[j]].z; }
                cx /= 5; cy /= 5; cz /= 5;
                float a11 = 0, a12 = 0, a13 = 0, a22 = 0, a23 = 0, a33 = 0;
                for (int j = 0; j < 5; j++) {
                    float ax = M[ind[j]].x - cx, ay = M[ind[j]].y - cy, az = M[ind[j]].z - cz;
                    a11 += ax * ax; a12 += ax * ay; a13 += ax * az;
                    a22 += ay * ay; a23 += ay * az;
                    a33 += az * az;
                }
                a11 /= 5; a12 /= 5; a13 /= 5; a22 /= 5; a23 /= 5; a33 /= 5;
                float A1[9] = {a11, a12, a13, a12, a22, a23, a13, a23, a33}, D1[3], V1[9];
                cv_eigen_sym(A1, 3, D1, V1);
                if (D1[0] > 3 * D1[1]) {
                    float x0 = pointSel.x, y0 = pointSel.y, z0 = pointSel.z;
                    float x1 = (float)(cx + 0.1 * V1[0]), y1 = (float)(cy + 0.1 * V1[1]), z1 = (float)(cz + 0.1 * V1[2]);
                    float x2 = (float)(cx - 0.1 * V1[0]), y2 = (float)(cy - 0.1 * V1[1]), z2 = (float)(cz - 0.1 * V1[2]);
                    float a012 = sqrtf(((x0 - x1) * (y0 - y2) - (x0 - x2) * (y0 - y1)) * ((x0 - x1) * (y0 - y2) - (x0 - x2) * (y0 - y1)) +
                                       ((x0 - x1) * (z0 - z2) - (x0 - x2) * (z0 - z1)) * ((x0 - x1) * (z0 - z2) - (x0 - x2) * (z0 - z1)) +
                                       ((y0 - y1) * (z0 - z2) - (y0 - y2) * (z0 - z1)) * ((y0 - y1) * (z0 - z2) - (y0 - y2) * (z0 - z1)));
                    float l12 = sqrtf((x1 - x2) * (x1 - x2) + (y1 - y2) * (y1 - y2) + (z1 - z2) * (z1 - z2));
                    float la = ((y1 - y2) * ((x0 - x1) * (y0 - y2) - (x0 - x2) * (y0 - y1)) +
                                (z1 - z2) * ((x0 - x1) * (z0 - z2) - (x0 - x2) * (z0 - z1))) / a012 / l12;
                    float lb = -((x1 - x2) * ((x0 - x1) * (y0 - y2) - (x0 - x2) * (y0 - y1)) -
                                 (z1 - z2) * ((y0 - y1) * (z0 - z2) - (y0 - y2) * (z0 - z1))) / a012 / l12;
                    float lc = -((x1 - x2) * ((x0 - x1) * (z0 - z2) - (x0 - x2) * (z0 - z1)) +
                                 (y1 - y2) * ((y0 - y1) * (z0 - z2) - (y0 - y2) * (z0 - z1))) / a012 / l12;
                    float ld2 = a012 / l12;
                    float s = (float)(1 - 0.9 * fabsf(ld2));
                    if (s > 0.1) {
                        laserCloudOri.push_back(pointOri);
                        coeffSel.push_back({s * la, s * lb, s * lc, s * ld2});
                    }
                }
            }
        }
    }

    void surfOptimization(int) {
        updatePointAssociateToMapSinCos();
        int ind[5]; float dis[5];
        const int mapN = (int)laserCloudSurfFromMapDS.size();
        for (size_t i = 0; i < laserCloudSurfTotalLastDS.size(); i++) {
            const Pt& pointOri = laserCloudSurfTotalLastDS[i];
            Pt pointSel = pointAssociateToMap(pointOri);
            int cnt = kdtreeSurfFromMap.knn(pointSel, 5, ind, dis);
            if (cnt < 5 || mapN < 5) continue;
            if (dis[4] < 1.0) {
                const Cloud& M = laserCloudSurfFromMapDS;
                float A0[15], B0[5] = {-1, -1, -1, -1, -1}, X0[3];
                for (int j = 0; j < 5; j++) { A0[j * 3] = M[ind[j]].x; A0[j * 3 + 1] = M[ind[j]].y; A0[j * 3 + 2] = M[ind[j]].z; }
                cv_solve_qr(A0, B0, 5, 3, X0);
                float pa = X0[0], pb = X0[1], pc = X0[2], pd = 1;
                float ps = sqrtf(pa * pa + pb * pb + pc * pc);
                pa /= ps; pb /= ps; pc /= ps; pd /= ps;
                bool planeValid = true;
                for (int j = 0; j < 5; j++) {
                    if (fabsf(pa * M[ind[j]].x + pb * M[ind[j]].y + pc * M[ind[j]].z + pd) > 0.2) { planeValid = false; break; }
                }
                if (planeValid) {
                    float pd2 = pa * pointSel.x + pb * pointSel.y + pc * pointSel.z + pd;
                    float s = (float)(1 - 0.9 * fabsf(pd2) /
                                              sqrtf(sqrtf(pointSel.x * pointSel.x + pointSel.y * pointSel.y + pointSel.z * pointSel.z)));
                    if (s > 0.1) {
                        laserCloudOri.push_back(pointOri);
                        coeffSel.push_back({s * pa, s * pb, s * pc, s * pd2});
                    }
                }
            }
        }
    }

    bool LMOptimization(int iterCount) {
        using namespace oracle_libm;
        float srx = sinf_(transformTobeMapped[0]), crx = cosf_(transformTobeMapped[0]);
        float sry = sinf_(transformTobeMapped[1]), cry = cosf_(transformTobeMapped[1]);
        float srz = sinf_(transformTobeMapped[2]), crz = cosf_(transformTobeMapped[2]);
        int n = (int)laserCloudOri.size();
        if (n < 50) return false;
        std::vector<float> A(n * 6), B(n);
        for (int i = 0; i < n; i++) {
            const Pt& p = laserCloudOri[i];
            const Pt& cf = coeffSel[i];
            float arx = (crx * sry * srz * p.x + crx * crz * sry * p.y - srx * sry * p.z) * cf.x +
                        (-srx * srz * p.x - crz * srx * p.y - crx * p.z) * cf.y +
                        (crx * cry * srz * p.x + crx * cry * crz * p.y - cry * srx * p.z) * cf.z;
            float ary = ((cry * srx * srz - crz * sry) * p.x + (sry * srz + cry * crz * srx) * p.y + crx * cry * p.z) * cf.x +
                        ((-cry * crz - srx * sry * srz) * p.x + (cry * srz - crz * srx * sry) * p.y - crx * sry * p.z) * cf.z;
            float arz = ((crz * srx * sry - cry * srz) * p.x + (-cry * crz - srx * sry * srz) * p.y) * cf.x +
                        (crx * crz * p.x - crx * srz * p.y) * cf.y +
                        ((sry * srz + cry * crz * srx) * p.x + (crz * sry - cry * srx * srz) * p.y) * cf.z;
            A[i * 6 + 0] = arx; A[i * 6 + 1] = ary; A[i * 6 + 2] = arz;
            A[i * 6 + 3] = cf.x; A[i * 6 + 4] = cf.y; A[i * 6 + 5] = cf.z;
            B[i] = -cf.intensity;
        }
        float AtA[36], AtB[6], X[6];
        gemm_AtA(A, n, 6, AtA);
        gemm_AtB(A, B, n, 6, AtB);
        cv_solve_qr(AtA, AtB, 6, 6, X);
        if (iterCount == 0) {
            float E[6], V[36], V2[36], Vi[36];
            cv_eigen_sym(AtA, 6, E, V);
            memcpy(V2, V, sizeof(V));
            isDegenerate = false;
            for (int i = 5; i >= 0; i--) {
                if (E[i] < 100) {
                    for (int j = 0; j < 6; j++) V2[i * 6 + j] = 0;
                    isDegenerate = true;
                } else break;
            }
            cv_inv(V, 6, Vi);
            gemm_small(Vi, V2, 6, 6, 6, matP);
        }
        if (isDegenerate) {
            float X2[6];
            memcpy(X2, X, sizeof(X2));
            gemm_small(matP, X2, 6, 6, 1, X);
        }
        for (int i = 0; i < 6; ++i) transformTobeMapped[i] += X[i];
        // pcl::rad2deg(float) = alpha * 57.29578f
        double r0 = X[0] * 57.29578f, r1 = X[1] * 57.29578f, r2 = X[2] * 57.29578f;
        double t0 = X[3] * 100, t1 = X[4] * 100, t2 = X[5] * 100;
        float deltaR = (float)sqrt(r0 * r0 + r1 * r1 + r2 * r2);
        float deltaT = (float)sqrt(t0 * t0 + t1 * t1 + t2 * t2);
        return deltaR < 0.05 && deltaT < 0.05;
    }

    void scan2MapOptimization() {
        lm_iters = 0;
        if ((int)laserCloudCornerFromMapDS.size() > 10 && (int)laserCloudSurfFromMapDS.size() > 100) {
            kdtreeCornerFromMap.build(laserCloudCornerFromMapDS);
            kdtreeSurfFromMap.build(laserCloudSurfFromMapDS);
            for (int iterCount = 0; iterCount < 10; iterCount++) {
                laserCloudOri.clear(); coeffSel.clear();
                cornerOptimization(iterCount);
                surfOptimization(iterCount);
                lm_iters = iterCount + 1;
                if (LMOptimization(iterCount)) break;
            }
            transformUpdate();
        }
    }

    void saveKeyFramesAndFactor() {
        saved_keyframe = false;
        currentRobotPosPoint.x = transformAftMapped[3];
        currentRobotPosPoint.y = transformAftMapped[4];
        currentRobotPosPoint.z = transformAftMapped[5];
        bool saveThisKeyFrame = true;
        float dx = previousRobotPosPoint.x - currentRobotPosPoint.x;
        float dy = previousRobotPosPoint.y - currentRobotPosPoint.y;
        float dz = previousRobotPosPoint.z - currentRobotPosPoint.z;
        if (sqrtf(dx * dx + dy * dy + dz * dz) < 0.3) saveThisKeyFrame = false;
        if (!saveThisKeyFrame && !keyPoses.empty()) return;
        previousRobotPosPoint = currentRobotPosPoint;
        // iSAM2 estimate of the new node == its initial value, read back
        // through Rot3::RzRyRx -> pitch()/yaw()/roll() (oracle_tf.h)
        float est[6];
        for (int i = 0; i < 6; ++i) kfPre[i] = keyPoses.empty() ? transformTobeMapped[i] : transformAftMapped[i];
        if (keyPoses.empty()) {
            for (int i = 0; i < 6; ++i) transformLast[i] = transformTobeMapped[i];
            keyframe_estimate(transformTobeMapped, est);
        } else {
            keyframe_estimate(transformAftMapped, est);
        }
        Pose6 p6{est[3], est[4], est[5], est[0], est[1], est[2]};
        keyPoses.push_back(p6);
        keyTimes.push_back(timeLaserOdometry);
        if (keyPoses.size() > 1) {
            float e[6];
            memcpy(e, est, sizeof(e));
            for (int i = 0; i < 6; ++i) { transformAftMapped[i] = e[i]; transformLast[i] = e[i]; transformTobeMapped[i] = e[i]; }
        }
        cornerCloudKeyFrames.push_back(laserCloudCornerLastDS);
        surfCloudKeyFrames.push_back(laserCloudSurfLastDS);
        outlierCloudKeyFrames.push_back(laserCloudOutlierLastDS);
        sc.makeAndSaveScancontextAndKeys(laserCloudRawDS);
        saved_keyframe = true;
    }

    // laserOdometryHandler + run() for one mapping opportunity.
    // raw: (x,y,z,i) x n_raw (NaNs included; VoxelGrid skips them: is_dense false)
    bool run(const Cloud& corner, const Cloud& surf, const Cloud& outlier, const float* odomSum,
             const float* raw, int n_raw, double t) {
        ran = false;
        saved_keyframe = false;
        odom_handoff(odomSum, transformSum);   // tf quaternion round trip (FA:1728 -> MO:658-666, Q18)
        timeLaserOdometry = t;
        if (!(t - timeLastProcessing >= cfg.mapping_process_interval)) return false;
        timeLastProcessing = t;
        laserCloudCornerLast = corner;
        laserCloudSurfLast = surf;
        laserCloudOutlierLast = outlier;
        laserCloudRaw.clear();
        for (int i = 0; i < n_raw; ++i) {
            const float* p = raw + 4 * (size_t)i;
            if (std::isfinite(p[0]) && std::isfinite(p[1]) && std::isfinite(p[2]))
                laserCloudRaw.push_back({p[0], p[1], p[2], p[3]});
        }
        ran = true;
        transformAssociateToMap();
        extractSurroundingKeyFrames();
        downsampleCurrentScan();
        scan2MapOptimization();
        saveKeyFramesAndFactor();
        odom_handoff(transformAftMapped, tfAft);   // publishTF: quaternion round trip (orientation)
        for (int k = 0; k < 6; ++k) tfBef[k] = transformBefMapped[k];   // twist fields, exact
        // clearCloud (MO:1640): the DS maps are kept aside for parity checks
        lastCornerMapDS.swap(laserCloudCornerFromMapDS);
        lastSurfMapDS.swap(laserCloudSurfFromMapDS);
        lastCornerMapRaw.swap(laserCloudCornerFromMap); lastSurfMapRaw.swap(laserCloudSurfFromMap);
        laserCloudCornerFromMap.clear(); laserCloudSurfFromMap.clear();
        laserCloudCornerFromMapDS.clear(); laserCloudSurfFromMapDS.clear();
        return true;
    }
};

}  // namespace oracle
