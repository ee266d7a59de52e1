// oracle_ip.h — TEST INFRASTRUCTURE ONLY: CPU restatement of
// imageProjection.cpp:145-460 (ImageProjection::cloudHandler minus ROS
// publishing).  Follows the reference line by line, including the quirks of
// Q1 (float -> size_t row truncation), Q2 (last point
// wins), Q3 (BFS row count excludes the seed), Q15 (ground overwrite order).
// Math is the host glibc's own atan2f / sinf / cosf (oracle_libm.h), which is
// what `using namespace std` resolves to in the reference.
#pragma once

#include "oracle_common.h"
#include "../sc-lego-loam_amd/csrc/slo_config.h"
#include "oracle_libm.h"

namespace oracle {

// cloud_info.msg:1-12
struct SegInfo {
    std::vector<int32_t> startRingIndex, endRingIndex;
    float startOrientation = 0, endOrientation = 0, orientationDiff = 0;
    std::vector<uint8_t> segmentedCloudGroundFlag;
    std::vector<uint32_t> segmentedCloudColInd;
    std::vector<float> segmentedCloudRange;
};

struct ImageProjection {
    slo_config cfg;
    int R, C;
    std::vector<float> rangeMat;   // R*C
    std::vector<int8_t> groundMat;
    std::vector<int32_t> labelMat;
    int labelCount = 1;
    Cloud fullCloud, fullInfoCloud, laserCloudIn;
    Cloud segmentedCloud, outlierCloud;
    SegInfo segMsg;
    std::vector<uint16_t> allPushedIndX, allPushedIndY, queueIndX, queueIndY;

    explicit ImageProjection(const slo_config& c) : cfg(c), R(c.n_scan), C(c.horizon_scan) {
        fullCloud.resize(R * C);
        fullInfoCloud.resize(R * C);
        segMsg.startRingIndex.assign(R, 0);
        segMsg.endRingIndex.assign(R, 0);
        segMsg.segmentedCloudGroundFlag.assign(R * C, 0);
        segMsg.segmentedCloudColInd.assign(R * C, 0);
        segMsg.segmentedCloudRange.assign(R * C, 0);
        allPushedIndX.resize(R * C); allPushedIndY.resize(R * C);
        queueIndX.resize(R * C); queueIndY.resize(R * C);
        resetParameters();
    }

    void resetParameters() {  // IP:145-159
        laserCloudIn.clear();
        segmentedCloud.clear();
        outlierCloud.clear();
        rangeMat.assign(R * C, FLT_MAX);
        groundMat.assign(R * C, 0);
        labelMat.assign(R * C, 0);
        labelCount = 1;
        const float qn = std::numeric_limits<float>::quiet_NaN();
        Pt nanPoint{qn, qn, qn, -1};
        std::fill(fullCloud.begin(), fullCloud.end(), nanPoint);
        std::fill(fullInfoCloud.begin(), fullInfoCloud.end(), nanPoint);
    }

    std::vector<uint16_t> rings;   // useCloudRing: the message's ring field, unfiltered order

    // IP:163-179 — removeNaNFromPointCloud keeps order; input is (x,y,z,i) x n
    void copyPointCloud(const float* pts, int n) {
        laserCloudIn.clear();
        for (int i = 0; i < n; ++i) {
            const float* p = pts + 4 * (size_t)i;
            if (!std::isfinite(p[0]) || !std::isfinite(p[1]) || !std::isfinite(p[2])) continue;
            laserCloudIn.push_back({p[0], p[1], p[2], p[3]});
        }
    }

    void findStartEndAngle() {  // IP:199-209
        const Pt& f = laserCloudIn.front();
        const Pt& l = laserCloudIn.back();
        segMsg.startOrientation = -oracle_libm::atan2f_(f.y, f.x);
        segMsg.endOrientation = (float)(-oracle_libm::atan2f_(l.y, l.x) + 2 * M_PI);
        if (segMsg.endOrientation - segMsg.startOrientation > 3 * M_PI)
            segMsg.endOrientation = (float)(segMsg.endOrientation - 2 * M_PI);
        else if (segMsg.endOrientation - segMsg.startOrientation < M_PI)
            segMsg.endOrientation = (float)(segMsg.endOrientation + 2 * M_PI);
        segMsg.orientationDiff = segMsg.endOrientation - segMsg.startOrientation;
    }

    void projectPointCloud() {  // IP:211-257
        size_t cloudSize = laserCloudIn.size();
        for (size_t i = 0; i < cloudSize; ++i) {
            Pt thisPoint = laserCloudIn[i];
            int64_t rowIdn;
            if (cfg.use_cloud_ring) {
                // IP:225-226: the ring of laserCloudInRing->points[i], the
                // UNfiltered cloud indexed by the filtered index i (the
                // reference requires is_dense clouds, IP:174-177)
                rowIdn = i < rings.size() ? (int64_t)rings[i] : 0;
            } else {
                float verticalAngle = (float)((double)(oracle_libm::atan2f_(thisPoint.z,
                    sqrtf(thisPoint.x * thisPoint.x + thisPoint.y * thisPoint.y)) * 180) / M_PI);
                float rowf = (verticalAngle + cfg.ang_bottom) / cfg.ang_res_y;
                // Q1: float -> size_t; negative values in (-1, 0) truncate to 0,
                // below -1 wrap to huge and are rejected by the range check.
                rowIdn = (int64_t)rowf;  // truncation toward zero
            }
            if (rowIdn < 0 || rowIdn >= R) continue;
            float horizonAngle = (float)((double)(oracle_libm::atan2f_(thisPoint.x, thisPoint.y) * 180) / M_PI);
            double colD = -round(((double)horizonAngle - 90.0) / (double)cfg.ang_res_x) + (double)(C / 2);
            int64_t columnIdn = (int64_t)colD;
            if (columnIdn >= C) columnIdn -= C;
            if (columnIdn < 0 || columnIdn >= C) continue;
            float range = sqrtf(thisPoint.x * thisPoint.x + thisPoint.y * thisPoint.y + thisPoint.z * thisPoint.z);
            if (range < cfg.sensor_minimum_range) continue;
            rangeMat[rowIdn * C + columnIdn] = range;
            // (float)rowIdn + (float)columnIdn / 10000.0 is evaluated in double
            thisPoint.intensity = (float)((double)(float)rowIdn + (double)(float)columnIdn / 10000.0);
            size_t index = columnIdn + rowIdn * C;
            fullCloud[index] = thisPoint;
            fullInfoCloud[index] = thisPoint;
            fullInfoCloud[index].intensity = range;
        }
    }

    void groundRemoval() {  // IP:260-310
        for (int j = 0; j < C; ++j) {
            for (int i = 0; i < cfg.ground_scan_ind; ++i) {
                size_t lowerInd = j + (i)*C;
                size_t upperInd = j + (i + 1) * C;
                if (fullCloud[lowerInd].intensity == -1 || fullCloud[upperInd].intensity == -1) {
                    groundMat[i * C + j] = -1;
                    continue;
                }
                float diffX = fullCloud[upperInd].x - fullCloud[lowerInd].x;
                float diffY = fullCloud[upperInd].y - fullCloud[lowerInd].y;
                float diffZ = fullCloud[upperInd].z - fullCloud[lowerInd].z;
                float angle = (float)((double)(oracle_libm::atan2f_(diffZ, sqrtf(diffX * diffX + diffY * diffY)) * 180) / M_PI);
                if (fabsf(angle - cfg.sensor_mount_angle) <= 10) {
                    groundMat[i * C + j] = 1;
                    groundMat[(i + 1) * C + j] = 1;
                }
            }
        }
        for (int i = 0; i < R; ++i)
            for (int j = 0; j < C; ++j)
                if (groundMat[i * C + j] == 1 || rangeMat[i * C + j] == FLT_MAX) labelMat[i * C + j] = -1;
    }

    void labelComponents(int row, int col) {  // IP:370-460
        std::vector<uint8_t> lineCountFlag(R, 0);
        queueIndX[0] = row; queueIndY[0] = col;
        int queueSize = 1, queueStartInd = 0, queueEndInd = 1;
        allPushedIndX[0] = row; allPushedIndY[0] = col;
        int allPushedIndSize = 1;
        static const int nb[4][2] = {{-1, 0}, {0, 1}, {0, -1}, {1, 0}};
        while (queueSize > 0) {
            int fromIndX = queueIndX[queueStartInd];
            int fromIndY = queueIndY[queueStartInd];
            --queueSize; ++queueStartInd;
            labelMat[fromIndX * C + fromIndY] = labelCount;
            for (int it = 0; it < 4; ++it) {
                int thisIndX = fromIndX + nb[it][0];
                int thisIndY = fromIndY + nb[it][1];
                if (thisIndX < 0 || thisIndX >= R) continue;
                if (thisIndY < 0) thisIndY = C - 1;
                if (thisIndY >= C) thisIndY = 0;
                if (labelMat[thisIndX * C + thisIndY] != 0) continue;
                float r1 = rangeMat[fromIndX * C + fromIndY], r2 = rangeMat[thisIndX * C + thisIndY];
                float d1 = std::max(r1, r2), d2 = std::min(r1, r2);
                float sa, ca;
                if (nb[it][0] == 0) { sa = cfg.sin_alpha_x; ca = cfg.cos_alpha_x; }
                else { sa = cfg.sin_alpha_y; ca = cfg.cos_alpha_y; }
                float angle = oracle_libm::atan2f_(d2 * sa, (d1 - d2 * ca));
                if (angle > cfg.segment_theta) {
                    queueIndX[queueEndInd] = thisIndX; queueIndY[queueEndInd] = thisIndY;
                    ++queueSize; ++queueEndInd;
                    labelMat[thisIndX * C + thisIndY] = labelCount;
                    lineCountFlag[thisIndX] = 1;
                    allPushedIndX[allPushedIndSize] = thisIndX;
                    allPushedIndY[allPushedIndSize] = thisIndY;
                    ++allPushedIndSize;
                }
            }
        }
        bool feasibleSegment = false;
        if (allPushedIndSize >= 30) feasibleSegment = true;
        else if (allPushedIndSize >= cfg.segment_valid_point_num) {
            int lineCount = 0;
            for (int i = 0; i < R; ++i) if (lineCountFlag[i]) ++lineCount;
            if (lineCount >= cfg.segment_valid_line_num) feasibleSegment = true;
        }
        if (feasibleSegment) ++labelCount;
        else
            for (int i = 0; i < allPushedIndSize; ++i)
                labelMat[allPushedIndX[i] * C + allPushedIndY[i]] = 999999;
    }

    void cloudSegmentation() {  // IP:312-368
        for (int i = 0; i < R; ++i)
            for (int j = 0; j < C; ++j)
                if (labelMat[i * C + j] == 0) labelComponents(i, j);
        int sizeOfSegCloud = 0;
        for (int i = 0; i < R; ++i) {
            segMsg.startRingIndex[i] = sizeOfSegCloud - 1 + 5;
            for (int j = 0; j < C; ++j) {
                int lab = labelMat[i * C + j];
                bool gnd = groundMat[i * C + j] == 1;
                if (lab > 0 || gnd) {
                    if (lab == 999999) {
                        if (i > cfg.ground_scan_ind && j % 5 == 0) outlierCloud.push_back(fullCloud[j + i * C]);
                        continue;
                    }
                    if (gnd) {
                        if (j % 5 != 0 && j > 5 && j < C - 5) continue;
                    }
                    segMsg.segmentedCloudGroundFlag[sizeOfSegCloud] = gnd;
                    segMsg.segmentedCloudColInd[sizeOfSegCloud] = j;
                    segMsg.segmentedCloudRange[sizeOfSegCloud] = rangeMat[i * C + j];
                    segmentedCloud.push_back(fullCloud[j + i * C]);
                    ++sizeOfSegCloud;
                }
            }
            segMsg.endRingIndex[i] = sizeOfSegCloud - 1 - 5;
        }
    }

    // cloudHandler (IP:181-197) minus publish; the caller reads outputs
    // before the next call (resetParameters happens at the start here, which
    // is equivalent because every reset field is only read after it).
    void cloudHandler(const float* pts, int n) {
        resetParameters();
        copyPointCloud(pts, n);
        // An empty cloud (no finite point) makes the reference read points[0]
        // of an empty vector (IP:201: undefined).  Defined here, as in the
        // GPU path: the orientations keep their previous values and every
        // other stage runs on an image with no returns.
        if (!laserCloudIn.empty()) findStartEndAngle();
        projectPointCloud();
        groundRemoval();
        cloudSegmentation();
    }
};

}  // namespace oracle
