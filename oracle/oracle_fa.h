// oracle_fa.h — TEST INFRASTRUCTURE ONLY: CPU restatement of
// featureAssociation.cpp: adjustDistortion 491-619 with its IMU branch,
// calculateSmoothness 621-641, markOccludedPoints 643-678, extractFeatures
// 680-784, TransformToStart/End 860-953, PluginIMURotation 955-1013,
// AccumulateRotation 1015-1032, correspondence search 1044-1268, the two
// 3-DOF solvers 1270-1478, checkSystemInitialization 1605-1637,
// updateTransformation 1666-1695, integrateTransformation 1697-1725,
// adjustOutlierCloud 1746-1757, publishCloudsLast 1759-1815, and the IMU
// path: imuHandler 459-486, AccumulateIMUShiftAndRotation 417-457,
// VeloToStartIMU 349-365, TransformToStartIMU 367-392, updateInitialGuess
// 1639-1664.  Without IMU messages (imuPointerLast = -1) every imu* quantity
// stays at its initial value exactly as in the reference.
// Persistent per-scan arrays (cloudCurvature, cloudNeighborPicked, cloudLabel,
// cloudSmoothness) keep their stale contents across scans (Appendix A Q5).
#pragma once

#include "oracle_ip.h"
#include "oracle_tf.h"

namespace oracle {

struct Smooth { float value; size_t ind; };

// sensor_msgs/Imu as imuHandler reads it (the layout of slo_imu_msg)
struct ImuMsg { double stamp, qx, qy, qz, qw, ax, ay, az, wx, wy, wz; };
constexpr int imuQueLength = 200;   // utility.h:113

struct FeatureAssociation {
    slo_config cfg;
    int R, C;
    // features state
    std::vector<Smooth> cloudSmoothness;
    std::vector<float> cloudCurvature;
    std::vector<int> cloudNeighborPicked, cloudLabel;
    Cloud segmentedCloud, outlierCloud;
    SegInfo segInfo;
    Cloud cornerPointsSharp, cornerPointsLessSharp, surfPointsFlat, surfPointsLessFlat;
    bool stable_voxel = false;
    // odometry state
    bool systemInitedLM = false;
    int frameCount;
    float transformCur[6] = {0, 0, 0, 0, 0, 0};
    float transformSum[6] = {0, 0, 0, 0, 0, 0};
    Cloud laserCloudCornerLast, laserCloudSurfLast, laserCloudOri, coeffSel;
    KdTree kdtreeCornerLast, kdtreeSurfLast;
    int laserCloudCornerLastNum = 0, laserCloudSurfLastNum = 0;
    std::vector<float> pointSearchCornerInd1, pointSearchCornerInd2;
    std::vector<float> pointSearchSurfInd1, pointSearchSurfInd2, pointSearchSurfInd3;
    bool isDegenerate = false;
    float matP[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0};
    // imu quantities (initializationValue, FA:249-295)
    double timeScanCur = 0;
    int imuPointerFront = 0, imuPointerLast = -1, imuPointerLastIteration = 0;
    float imuRollStart = 0, imuPitchStart = 0, imuYawStart = 0;
    float cosImuRollStart = 0, cosImuPitchStart = 0, cosImuYawStart = 0;
    float sinImuRollStart = 0, sinImuPitchStart = 0, sinImuYawStart = 0;
    float imuRollCur = 0, imuPitchCur = 0, imuYawCur = 0;
    float imuVeloXStart = 0, imuVeloYStart = 0, imuVeloZStart = 0;
    float imuShiftXStart = 0, imuShiftYStart = 0, imuShiftZStart = 0;
    float imuVeloXCur = 0, imuVeloYCur = 0, imuVeloZCur = 0;
    float imuShiftXCur = 0, imuShiftYCur = 0, imuShiftZCur = 0;
    float imuShiftFromStartXCur = 0, imuShiftFromStartYCur = 0, imuShiftFromStartZCur = 0;
    float imuVeloFromStartXCur = 0, imuVeloFromStartYCur = 0, imuVeloFromStartZCur = 0;
    float imuAngularRotationXCur = 0, imuAngularRotationYCur = 0, imuAngularRotationZCur = 0;
    float imuAngularRotationXLast = 0, imuAngularRotationYLast = 0, imuAngularRotationZLast = 0;
    float imuAngularFromStartX = 0, imuAngularFromStartY = 0, imuAngularFromStartZ = 0;
    double imuTime[imuQueLength] = {};
    float imuRoll[imuQueLength] = {}, imuPitch[imuQueLength] = {}, imuYaw[imuQueLength] = {};
    float imuAccX[imuQueLength] = {}, imuAccY[imuQueLength] = {}, imuAccZ[imuQueLength] = {};
    float imuVeloX[imuQueLength] = {}, imuVeloY[imuQueLength] = {}, imuVeloZ[imuQueLength] = {};
    float imuShiftX[imuQueLength] = {}, imuShiftY[imuQueLength] = {}, imuShiftZ[imuQueLength] = {};
    float imuAngularVeloX[imuQueLength] = {}, imuAngularVeloY[imuQueLength] = {}, imuAngularVeloZ[imuQueLength] = {};
    float imuAngularRotationX[imuQueLength] = {}, imuAngularRotationY[imuQueLength] = {},
          imuAngularRotationZ[imuQueLength] = {};
    float imuRollLast = 0, imuPitchLast = 0, imuYawLast = 0;
    float imuShiftFromStartX = 0, imuShiftFromStartY = 0, imuShiftFromStartZ = 0;
    float imuVeloFromStartX = 0, imuVeloFromStartY = 0, imuVeloFromStartZ = 0;
    // outputs of the last scan
    bool published_to_mapping = false;
    int iters_surf = 0, iters_corner = 0;

    explicit FeatureAssociation(const slo_config& c) : cfg(c), R(c.n_scan), C(c.horizon_scan) {
        size_t H = (size_t)R * C;
        cloudSmoothness.assign(H, Smooth{0.0f, 0});
        cloudCurvature.assign(H, 0.0f);   // new float[] — zero pages in practice
        cloudNeighborPicked.assign(H, 0);
        cloudLabel.assign(H, 0);
        pointSearchCornerInd1.assign(H, 0); pointSearchCornerInd2.assign(H, 0);
        pointSearchSurfInd1.assign(H, 0); pointSearchSurfInd2.assign(H, 0); pointSearchSurfInd3.assign(H, 0);
        frameCount = cfg.skip_frame_num;
    }

    // ------------------------------------------------------------ IMU
    void updateImuRollPitchYawStartSinCos() {
        using namespace oracle_libm;
        cosImuRollStart = cosf_(imuRollStart); cosImuPitchStart = cosf_(imuPitchStart); cosImuYawStart = cosf_(imuYawStart);
        sinImuRollStart = sinf_(imuRollStart); sinImuPitchStart = sinf_(imuPitchStart); sinImuYawStart = sinf_(imuYawStart);
    }

    void VeloToStartIMU() {
        imuVeloFromStartXCur = imuVeloXCur - imuVeloXStart;
        imuVeloFromStartYCur = imuVeloYCur - imuVeloYStart;
        imuVeloFromStartZCur = imuVeloZCur - imuVeloZStart;
        float x1 = cosImuYawStart * imuVeloFromStartXCur - sinImuYawStart * imuVeloFromStartZCur;
        float y1 = imuVeloFromStartYCur;
        float z1 = sinImuYawStart * imuVeloFromStartXCur + cosImuYawStart * imuVeloFromStartZCur;
        float x2 = x1;
        float y2 = cosImuPitchStart * y1 + sinImuPitchStart * z1;
        float z2 = -sinImuPitchStart * y1 + cosImuPitchStart * z1;
        imuVeloFromStartXCur = cosImuRollStart * x2 + sinImuRollStart * y2;
        imuVeloFromStartYCur = -sinImuRollStart * x2 + cosImuRollStart * y2;
        imuVeloFromStartZCur = z2;
    }

    void TransformToStartIMU(Pt* p) {
        using namespace oracle_libm;
        float x1 = cosf_(imuRollCur) * p->x - sinf_(imuRollCur) * p->y;
        float y1 = sinf_(imuRollCur) * p->x + cosf_(imuRollCur) * p->y;
        float z1 = p->z;
        float x2 = x1;
        float y2 = cosf_(imuPitchCur) * y1 - sinf_(imuPitchCur) * z1;
        float z2 = sinf_(imuPitchCur) * y1 + cosf_(imuPitchCur) * z1;
        float x3 = cosf_(imuYawCur) * x2 + sinf_(imuYawCur) * z2;
        float y3 = y2;
        float z3 = -sinf_(imuYawCur) * x2 + cosf_(imuYawCur) * z2;
        float x4 = cosImuYawStart * x3 - sinImuYawStart * z3;
        float y4 = y3;
        float z4 = sinImuYawStart * x3 + cosImuYawStart * z3;
        float x5 = x4;
        float y5 = cosImuPitchStart * y4 + sinImuPitchStart * z4;
        float z5 = -sinImuPitchStart * y4 + cosImuPitchStart * z4;
        p->x = cosImuRollStart * x5 + sinImuRollStart * y5 + imuShiftFromStartXCur;
        p->y = -sinImuRollStart * x5 + cosImuRollStart * y5 + imuShiftFromStartYCur;
        p->z = z5 + imuShiftFromStartZCur;
    }

    void AccumulateIMUShiftAndRotation() {
        using namespace oracle_libm;
        float roll = imuRoll[imuPointerLast];
        float pitch = imuPitch[imuPointerLast];
        float yaw = imuYaw[imuPointerLast];
        float accX = imuAccX[imuPointerLast];
        float accY = imuAccY[imuPointerLast];
        float accZ = imuAccZ[imuPointerLast];
        float x1 = cosf_(roll) * accX - sinf_(roll) * accY;
        float y1 = sinf_(roll) * accX + cosf_(roll) * accY;
        float z1 = accZ;
        float x2 = x1;
        float y2 = cosf_(pitch) * y1 - sinf_(pitch) * z1;
        float z2 = sinf_(pitch) * y1 + cosf_(pitch) * z1;
        accX = cosf_(yaw) * x2 + sinf_(yaw) * z2;
        accY = y2;
        accZ = -sinf_(yaw) * x2 + cosf_(yaw) * z2;
        int imuPointerBack = (imuPointerLast + imuQueLength - 1) % imuQueLength;
        double timeDiff = imuTime[imuPointerLast] - imuTime[imuPointerBack];
        if (timeDiff < cfg.scan_period) {
            imuShiftX[imuPointerLast] = imuShiftX[imuPointerBack] + imuVeloX[imuPointerBack] * timeDiff + accX * timeDiff * timeDiff / 2;
            imuShiftY[imuPointerLast] = imuShiftY[imuPointerBack] + imuVeloY[imuPointerBack] * timeDiff + accY * timeDiff * timeDiff / 2;
            imuShiftZ[imuPointerLast] = imuShiftZ[imuPointerBack] + imuVeloZ[imuPointerBack] * timeDiff + accZ * timeDiff * timeDiff / 2;
            imuVeloX[imuPointerLast] = imuVeloX[imuPointerBack] + accX * timeDiff;
            imuVeloY[imuPointerLast] = imuVeloY[imuPointerBack] + accY * timeDiff;
            imuVeloZ[imuPointerLast] = imuVeloZ[imuPointerBack] + accZ * timeDiff;
            imuAngularRotationX[imuPointerLast] = imuAngularRotationX[imuPointerBack] + imuAngularVeloX[imuPointerBack] * timeDiff;
            imuAngularRotationY[imuPointerLast] = imuAngularRotationY[imuPointerBack] + imuAngularVeloY[imuPointerBack] * timeDiff;
            imuAngularRotationZ[imuPointerLast] = imuAngularRotationZ[imuPointerBack] + imuAngularVeloZ[imuPointerBack] * timeDiff;
        }
    }

    void imuHandler(const ImuMsg& imuIn) {
        using namespace oracle_libm;
        double roll, pitch, yaw;
        tf_get_rpy(TfQuat{imuIn.qx, imuIn.qy, imuIn.qz, imuIn.qw}, roll, pitch, yaw);
        float accX = imuIn.ay - sin_d(roll) * cos_d(pitch) * 9.81;
        float accY = imuIn.az - cos_d(roll) * cos_d(pitch) * 9.81;
        float accZ = imuIn.ax + sin_d(pitch) * 9.81;
        imuPointerLast = (imuPointerLast + 1) % imuQueLength;
        imuTime[imuPointerLast] = imuIn.stamp;
        imuRoll[imuPointerLast] = roll;
        imuPitch[imuPointerLast] = pitch;
        imuYaw[imuPointerLast] = yaw;
        imuAccX[imuPointerLast] = accX;
        imuAccY[imuPointerLast] = accY;
        imuAccZ[imuPointerLast] = accZ;
        imuAngularVeloX[imuPointerLast] = imuIn.wx;
        imuAngularVeloY[imuPointerLast] = imuIn.wy;
        imuAngularVeloZ[imuPointerLast] = imuIn.wz;
        AccumulateIMUShiftAndRotation();
    }

    // ------------------------------------------------------------ features
    void adjustDistortion() {
        bool halfPassed = false;
        int cloudSize = (int)segmentedCloud.size();
        for (int i = 0; i < cloudSize; i++) {
            Pt point;
            point.x = segmentedCloud[i].y;
            point.y = segmentedCloud[i].z;
            point.z = segmentedCloud[i].x;
            float ori = -oracle_libm::atan2f_(point.x, point.z);
            if (!halfPassed) {
                if (ori < segInfo.startOrientation - M_PI / 2) ori = (float)(ori + 2 * M_PI);
                else if (ori > segInfo.startOrientation + M_PI * 3 / 2) ori = (float)(ori - 2 * M_PI);
                if (ori - segInfo.startOrientation > M_PI) halfPassed = true;
            } else {
                ori = (float)(ori + 2 * M_PI);
                if (ori < segInfo.endOrientation - M_PI * 3 / 2) ori = (float)(ori + 2 * M_PI);
                else if (ori > segInfo.endOrientation + M_PI / 2) ori = (float)(ori - 2 * M_PI);
            }
            float relTime = (ori - segInfo.startOrientation) / segInfo.orientationDiff;
            point.intensity = (float)(int)segmentedCloud[i].intensity + cfg.scan_period * relTime;
            if (imuPointerLast >= 0) {
                float pointTime = relTime * cfg.scan_period;
                imuPointerFront = imuPointerLastIteration;
                while (imuPointerFront != imuPointerLast) {
                    if (timeScanCur + pointTime < imuTime[imuPointerFront]) break;
                    imuPointerFront = (imuPointerFront + 1) % imuQueLength;
                }
                if (timeScanCur + pointTime > imuTime[imuPointerFront]) {
                    imuRollCur = imuRoll[imuPointerFront];
                    imuPitchCur = imuPitch[imuPointerFront];
                    imuYawCur = imuYaw[imuPointerFront];
                    imuVeloXCur = imuVeloX[imuPointerFront];
                    imuVeloYCur = imuVeloY[imuPointerFront];
                    imuVeloZCur = imuVeloZ[imuPointerFront];
                    imuShiftXCur = imuShiftX[imuPointerFront];
                    imuShiftYCur = imuShiftY[imuPointerFront];
                    imuShiftZCur = imuShiftZ[imuPointerFront];
                } else {
                    int imuPointerBack = (imuPointerFront + imuQueLength - 1) % imuQueLength;
                    float ratioFront = (timeScanCur + pointTime - imuTime[imuPointerBack]) /
                                       (imuTime[imuPointerFront] - imuTime[imuPointerBack]);
                    float ratioBack = (imuTime[imuPointerFront] - timeScanCur - pointTime) /
                                      (imuTime[imuPointerFront] - imuTime[imuPointerBack]);
                    imuRollCur = imuRoll[imuPointerFront] * ratioFront + imuRoll[imuPointerBack] * ratioBack;
                    imuPitchCur = imuPitch[imuPointerFront] * ratioFront + imuPitch[imuPointerBack] * ratioBack;
                    if (imuYaw[imuPointerFront] - imuYaw[imuPointerBack] > M_PI) {
                        imuYawCur = imuYaw[imuPointerFront] * ratioFront + (imuYaw[imuPointerBack] + 2 * M_PI) * ratioBack;
                    } else if (imuYaw[imuPointerFront] - imuYaw[imuPointerBack] < -M_PI) {
                        imuYawCur = imuYaw[imuPointerFront] * ratioFront + (imuYaw[imuPointerBack] - 2 * M_PI) * ratioBack;
                    } else {
                        imuYawCur = imuYaw[imuPointerFront] * ratioFront + imuYaw[imuPointerBack] * ratioBack;
                    }
                    imuVeloXCur = imuVeloX[imuPointerFront] * ratioFront + imuVeloX[imuPointerBack] * ratioBack;
                    imuVeloYCur = imuVeloY[imuPointerFront] * ratioFront + imuVeloY[imuPointerBack] * ratioBack;
                    imuVeloZCur = imuVeloZ[imuPointerFront] * ratioFront + imuVeloZ[imuPointerBack] * ratioBack;
                    imuShiftXCur = imuShiftX[imuPointerFront] * ratioFront + imuShiftX[imuPointerBack] * ratioBack;
                    imuShiftYCur = imuShiftY[imuPointerFront] * ratioFront + imuShiftY[imuPointerBack] * ratioBack;
                    imuShiftZCur = imuShiftZ[imuPointerFront] * ratioFront + imuShiftZ[imuPointerBack] * ratioBack;
                }
                if (i == 0) {
                    imuRollStart = imuRollCur;
                    imuPitchStart = imuPitchCur;
                    imuYawStart = imuYawCur;
                    imuVeloXStart = imuVeloXCur;
                    imuVeloYStart = imuVeloYCur;
                    imuVeloZStart = imuVeloZCur;
                    imuShiftXStart = imuShiftXCur;
                    imuShiftYStart = imuShiftYCur;
                    imuShiftZStart = imuShiftZCur;
                    if (timeScanCur + pointTime > imuTime[imuPointerFront]) {
                        imuAngularRotationXCur = imuAngularRotationX[imuPointerFront];
                        imuAngularRotationYCur = imuAngularRotationY[imuPointerFront];
                        imuAngularRotationZCur = imuAngularRotationZ[imuPointerFront];
                    } else {
                        int imuPointerBack = (imuPointerFront + imuQueLength - 1) % imuQueLength;
                        float ratioFront = (timeScanCur + pointTime - imuTime[imuPointerBack]) /
                                           (imuTime[imuPointerFront] - imuTime[imuPointerBack]);
                        float ratioBack = (imuTime[imuPointerFront] - timeScanCur - pointTime) /
                                          (imuTime[imuPointerFront] - imuTime[imuPointerBack]);
                        imuAngularRotationXCur = imuAngularRotationX[imuPointerFront] * ratioFront + imuAngularRotationX[imuPointerBack] * ratioBack;
                        imuAngularRotationYCur = imuAngularRotationY[imuPointerFront] * ratioFront + imuAngularRotationY[imuPointerBack] * ratioBack;
                        imuAngularRotationZCur = imuAngularRotationZ[imuPointerFront] * ratioFront + imuAngularRotationZ[imuPointerBack] * ratioBack;
                    }
                    imuAngularFromStartX = imuAngularRotationXCur - imuAngularRotationXLast;
                    imuAngularFromStartY = imuAngularRotationYCur - imuAngularRotationYLast;
                    imuAngularFromStartZ = imuAngularRotationZCur - imuAngularRotationZLast;
                    imuAngularRotationXLast = imuAngularRotationXCur;
                    imuAngularRotationYLast = imuAngularRotationYCur;
                    imuAngularRotationZLast = imuAngularRotationZCur;
                    updateImuRollPitchYawStartSinCos();
                } else {
                    VeloToStartIMU();
                    TransformToStartIMU(&point);
                }
            }
            segmentedCloud[i] = point;
        }
        imuPointerLastIteration = imuPointerLast;
    }

    void calculateSmoothness() {
        int cloudSize = (int)segmentedCloud.size();
        const float* r = segInfo.segmentedCloudRange.data();
        for (int i = 5; i < cloudSize - 5; i++) {
            float diffRange = r[i - 5] + r[i - 4] + r[i - 3] + r[i - 2] + r[i - 1] - r[i] * 10 +
                              r[i + 1] + r[i + 2] + r[i + 3] + r[i + 4] + r[i + 5];
            cloudCurvature[i] = diffRange * diffRange;
            cloudNeighborPicked[i] = 0;
            cloudLabel[i] = 0;
            cloudSmoothness[i].value = cloudCurvature[i];
            cloudSmoothness[i].ind = i;
        }
    }

    void markOccludedPoints() {
        int cloudSize = (int)segmentedCloud.size();
        const float* r = segInfo.segmentedCloudRange.data();
        const uint32_t* col = segInfo.segmentedCloudColInd.data();
        for (int i = 5; i < cloudSize - 6; ++i) {
            float depth1 = r[i], depth2 = r[i + 1];
            int columnDiff = std::abs((int)(col[i + 1] - col[i]));
            if (columnDiff < 10) {
                if (depth1 - depth2 > 0.3) {
                    for (int k = i - 5; k <= i; ++k) cloudNeighborPicked[k] = 1;
                } else if (depth2 - depth1 > 0.3) {
                    for (int k = i + 1; k <= i + 6; ++k) cloudNeighborPicked[k] = 1;
                }
            }
            float diff1 = fabsf((float)(r[i - 1] - r[i]));
            float diff2 = fabsf((float)(r[i + 1] - r[i]));
            if (diff1 > 0.02 * r[i] && diff2 > 0.02 * r[i]) cloudNeighborPicked[i] = 1;
        }
    }

    // segmentedCloudColInd[k] with the k = -1 read of a pick at ind = 4
    // (Appendix A Q5): the 4 bytes before the message vector's data are the
    // high half of glibc's chunk-size word, i.e. 0.
    uint32_t colAt(int k) const { return k < 0 ? 0u : segInfo.segmentedCloudColInd[k]; }
    void markPicked(int k) { if (k >= 0) cloudNeighborPicked[k] = 1; }

    void markNeighbors(int ind) {
        for (int l = 1; l <= 5; l++) {
            int columnDiff = std::abs((int)(colAt(ind + l) - colAt(ind + l - 1)));
            if (columnDiff > 10) break;
            markPicked(ind + l);
        }
        for (int l = -1; l >= -5; l--) {
            int columnDiff = std::abs((int)(colAt(ind + l) - colAt(ind + l + 1)));
            if (columnDiff > 10) break;
            markPicked(ind + l);
        }
    }

    void extractFeatures() {
        cornerPointsSharp.clear(); cornerPointsLessSharp.clear();
        surfPointsFlat.clear(); surfPointsLessFlat.clear();
        const int S = (int)segmentedCloud.size();
        Cloud lessFlatScan, lessFlatScanDS;
        for (int i = 0; i < R; i++) {
            lessFlatScan.clear();
            for (int j = 0; j < 6; j++) {
                int sp = (segInfo.startRingIndex[i] * (6 - j) + segInfo.endRingIndex[i] * j) / 6;
                int ep = (segInfo.startRingIndex[i] * (5 - j) + segInfo.endRingIndex[i] * (j + 1)) / 6 - 1;
                if (sp >= ep) continue;
                std::sort(cloudSmoothness.begin() + sp, cloudSmoothness.begin() + ep,
                          [](const Smooth& a, const Smooth& b) { return a.value < b.value; });
                int largestPickedNum = 0;
                for (int k = ep; k >= sp; k--) {
                    int ind = (int)cloudSmoothness[k].ind;
                    if (ind >= S) continue;  // stale index beyond this scan (UB in the reference)
                    if (cloudNeighborPicked[ind] == 0 && cloudCurvature[ind] > cfg.edge_threshold &&
                        segInfo.segmentedCloudGroundFlag[ind] == 0) {
                        largestPickedNum++;
                        if (largestPickedNum <= 2) {
                            cloudLabel[ind] = 2;
                            cornerPointsSharp.push_back(segmentedCloud[ind]);
                            cornerPointsLessSharp.push_back(segmentedCloud[ind]);
                        } else if (largestPickedNum <= 20) {
                            cloudLabel[ind] = 1;
                            cornerPointsLessSharp.push_back(segmentedCloud[ind]);
                        } else {
                            break;
                        }
                        cloudNeighborPicked[ind] = 1;
                        markNeighbors(ind);
                    }
                }
                int smallestPickedNum = 0;
                for (int k = sp; k <= ep; k++) {
                    int ind = (int)cloudSmoothness[k].ind;
                    if (ind >= S) continue;
                    if (cloudNeighborPicked[ind] == 0 && cloudCurvature[ind] < cfg.surf_threshold &&
                        segInfo.segmentedCloudGroundFlag[ind] == 1) {
                        cloudLabel[ind] = -1;
                        surfPointsFlat.push_back(segmentedCloud[ind]);
                        smallestPickedNum++;
                        if (smallestPickedNum >= 4) break;
                        cloudNeighborPicked[ind] = 1;
                        markNeighbors(ind);
                    }
                }
                for (int k = sp; k <= ep; k++)
                    if (cloudLabel[k] <= 0) lessFlatScan.push_back(segmentedCloud[k]);
            }
            voxel_grid(lessFlatScan, cfg.leaf_less_flat, lessFlatScanDS, stable_voxel);
            surfPointsLessFlat.insert(surfPointsLessFlat.end(), lessFlatScanDS.begin(), lessFlatScanDS.end());
        }
    }

    // ------------------------------------------------------------ transforms
    void TransformToStart(const Pt& pi, Pt& po) const {
        using namespace oracle_libm;
        float s = 10 * (pi.intensity - (float)(int)pi.intensity);
        float rx = s * transformCur[0], ry = s * transformCur[1], rz = s * transformCur[2];
        float tx = s * transformCur[3], ty = s * transformCur[4], tz = s * transformCur[5];
        float x1 = cosf_(rz) * (pi.x - tx) + sinf_(rz) * (pi.y - ty);
        float y1 = -sinf_(rz) * (pi.x - tx) + cosf_(rz) * (pi.y - ty);
        float z1 = (pi.z - tz);
        float x2 = x1;
        float y2 = cosf_(rx) * y1 + sinf_(rx) * z1;
        float z2 = -sinf_(rx) * y1 + cosf_(rx) * z1;
        po.x = cosf_(ry) * x2 - sinf_(ry) * z2;
        po.y = y2;
        po.z = sinf_(ry) * x2 + cosf_(ry) * z2;
        po.intensity = pi.intensity;
    }

    void TransformToEnd(const Pt& pi, Pt& po) const {
        using namespace oracle_libm;
        float s = 10 * (pi.intensity - (float)(int)pi.intensity);
        float rx = s * transformCur[0], ry = s * transformCur[1], rz = s * transformCur[2];
        float tx = s * transformCur[3], ty = s * transformCur[4], tz = s * transformCur[5];
        float x1 = cosf_(rz) * (pi.x - tx) + sinf_(rz) * (pi.y - ty);
        float y1 = -sinf_(rz) * (pi.x - tx) + cosf_(rz) * (pi.y - ty);
        float z1 = (pi.z - tz);
        float x2 = x1;
        float y2 = cosf_(rx) * y1 + sinf_(rx) * z1;
        float z2 = -sinf_(rx) * y1 + cosf_(rx) * z1;
        float x3 = cosf_(ry) * x2 - sinf_(ry) * z2;
        float y3 = y2;
        float z3 = sinf_(ry) * x2 + cosf_(ry) * z2;
        rx = transformCur[0]; ry = transformCur[1]; rz = transformCur[2];
        tx = transformCur[3]; ty = transformCur[4]; tz = transformCur[5];
        float x4 = cosf_(ry) * x3 + sinf_(ry) * z3;
        float y4 = y3;
        float z4 = -sinf_(ry) * x3 + cosf_(ry) * z3;
        float x5 = x4;
        float y5 = cosf_(rx) * y4 - sinf_(rx) * z4;
        float z5 = sinf_(rx) * y4 + cosf_(rx) * z4;
        float x6 = cosf_(rz) * x5 - sinf_(rz) * y5 + tx;
        float y6 = sinf_(rz) * x5 + cosf_(rz) * y5 + ty;
        float z6 = z5 + tz;
        float x7 = cosImuRollStart * (x6 - imuShiftFromStartX) - sinImuRollStart * (y6 - imuShiftFromStartY);
        float y7 = sinImuRollStart * (x6 - imuShiftFromStartX) + cosImuRollStart * (y6 - imuShiftFromStartY);
        float z7 = z6 - imuShiftFromStartZ;
        float x8 = x7;
        float y8 = cosImuPitchStart * y7 - sinImuPitchStart * z7;
        float z8 = sinImuPitchStart * y7 + cosImuPitchStart * z7;
        float x9 = cosImuYawStart * x8 + sinImuYawStart * z8;
        float y9 = y8;
        float z9 = -sinImuYawStart * x8 + cosImuYawStart * z8;
        float x10 = cosf_(imuYawLast) * x9 - sinf_(imuYawLast) * z9;
        float y10 = y9;
        float z10 = sinf_(imuYawLast) * x9 + cosf_(imuYawLast) * z9;
        float x11 = x10;
        float y11 = cosf_(imuPitchLast) * y10 + sinf_(imuPitchLast) * z10;
        float z11 = -sinf_(imuPitchLast) * y10 + cosf_(imuPitchLast) * z10;
        po.x = cosf_(imuRollLast) * x11 + sinf_(imuRollLast) * y11;
        po.y = -sinf_(imuRollLast) * x11 + cosf_(imuRollLast) * y11;
        po.z = z11;
        po.intensity = (float)(int)pi.intensity;
    }

    static void PluginIMURotation(float bcx, float bcy, float bcz, float blx, float bly, float blz,
                                  float alx, float aly, float alz, float& acx, float& acy, float& acz) {
        using namespace oracle_libm;
        float sbcx = sinf_(bcx), cbcx = cosf_(bcx), sbcy = sinf_(bcy), cbcy = cosf_(bcy);
        float sbcz = sinf_(bcz), cbcz = cosf_(bcz);
        float sblx = sinf_(blx), cblx = cosf_(blx), sbly = sinf_(bly), cbly = cosf_(bly);
        float sblz = sinf_(blz), cblz = cosf_(blz);
        float salx = sinf_(alx), calx = cosf_(alx), saly = sinf_(aly), caly = cosf_(aly);
        float salz = sinf_(alz), calz = cosf_(alz);
        float srx = -sbcx * (salx * sblx + calx * caly * cblx * cbly + calx * cblx * saly * sbly) -
                    cbcx * cbcz * (calx * saly * (cbly * sblz - cblz * sblx * sbly) -
                                   calx * caly * (sbly * sblz + cbly * cblz * sblx) + cblx * cblz * salx) -
                    cbcx * sbcz * (calx * caly * (cblz * sbly - cbly * sblx * sblz) -
                                   calx * saly * (cbly * cblz + sblx * sbly * sblz) + cblx * salx * sblz);
        acx = -asinf_(srx);
        float srycrx = (cbcy * sbcz - cbcz * sbcx * sbcy) * (calx * saly * (cbly * sblz - cblz * sblx * sbly) -
                                                          calx * caly * (sbly * sblz + cbly * cblz * sblx) +
                                                          cblx * cblz * salx) -
                       (cbcy * cbcz + sbcx * sbcy * sbcz) * (calx * caly * (cblz * sbly - cbly * sblx * sblz) -
                                                          calx * saly * (cbly * cblz + sblx * sbly * sblz) +
                                                          cblx * salx * sblz) +
                       cbcx * sbcy * (salx * sblx + calx * caly * cblx * cbly + calx * cblx * saly * sbly);
        float crycrx = (cbcz * sbcy - cbcy * sbcx * sbcz) * (calx * caly * (cblz * sbly - cbly * sblx * sblz) -
                                                          calx * saly * (cbly * cblz + sblx * sbly * sblz) +
                                                          cblx * salx * sblz) -
                       (sbcy * sbcz + cbcy * cbcz * sbcx) * (calx * saly * (cbly * sblz - cblz * sblx * sbly) -
                                                          calx * caly * (sbly * sblz + cbly * cblz * sblx) +
                                                          cblx * cblz * salx) +
                       cbcx * cbcy * (salx * sblx + calx * caly * cblx * cbly + calx * cblx * saly * sbly);
        acy = atan2f_(srycrx / cosf_(acx), crycrx / cosf_(acx));
        float srzcrx = sbcx * (cblx * cbly * (calz * saly - caly * salx * salz) -
                               cblx * sbly * (caly * calz + salx * saly * salz) + calx * salz * sblx) -
                       cbcx * cbcz * ((caly * calz + salx * saly * salz) * (cbly * sblz - cblz * sblx * sbly) +
                                      (calz * saly - caly * salx * salz) * (sbly * sblz + cbly * cblz * sblx) -
                                      calx * cblx * cblz * salz) +
                       cbcx * sbcz * ((caly * calz + salx * saly * salz) * (cbly * cblz + sblx * sbly * sblz) +
                                      (calz * saly - caly * salx * salz) * (cblz * sbly - cbly * sblx * sblz) +
                                      calx * cblx * salz * sblz);
        float crzcrx = sbcx * (cblx * sbly * (caly * salz - calz * salx * saly) -
                               cblx * cbly * (saly * salz + caly * calz * salx) + calx * calz * sblx) +
                       cbcx * cbcz * ((saly * salz + caly * calz * salx) * (sbly * sblz + cbly * cblz * sblx) +
                                      (caly * salz - calz * salx * saly) * (cbly * sblz - cblz * sblx * sbly) +
                                      calx * calz * cblx * cblz) -
                       cbcx * sbcz * ((saly * salz + caly * calz * salx) * (cblz * sbly - cbly * sblx * sblz) +
                                      (caly * salz - calz * salx * saly) * (cbly * cblz + sblx * sbly * sblz) -
                                      calx * calz * cblx * sblz);
        acz = atan2f_(srzcrx / cosf_(acx), crzcrx / cosf_(acx));
    }

    static void AccumulateRotation(float cx, float cy, float cz, float lx, float ly, float lz,
                                   float& ox, float& oy, float& oz) {
        using namespace oracle_libm;
        float srx = cosf_(lx) * cosf_(cx) * sinf_(ly) * sinf_(cz) - cosf_(cx) * cosf_(cz) * sinf_(lx) -
                    cosf_(lx) * cosf_(ly) * sinf_(cx);
        ox = -asinf_(srx);
        float srycrx = sinf_(lx) * (cosf_(cy) * sinf_(cz) - cosf_(cz) * sinf_(cx) * sinf_(cy)) +
                       cosf_(lx) * sinf_(ly) * (cosf_(cy) * cosf_(cz) + sinf_(cx) * sinf_(cy) * sinf_(cz)) +
                       cosf_(lx) * cosf_(ly) * cosf_(cx) * sinf_(cy);
        float crycrx = cosf_(lx) * cosf_(ly) * cosf_(cx) * cosf_(cy) -
                       cosf_(lx) * sinf_(ly) * (cosf_(cz) * sinf_(cy) - cosf_(cy) * sinf_(cx) * sinf_(cz)) -
                       sinf_(lx) * (sinf_(cy) * sinf_(cz) + cosf_(cy) * cosf_(cz) * sinf_(cx));
        oy = atan2f_(srycrx / cosf_(ox), crycrx / cosf_(ox));
        float srzcrx = sinf_(cx) * (cosf_(lz) * sinf_(ly) - cosf_(ly) * sinf_(lx) * sinf_(lz)) +
                       cosf_(cx) * sinf_(cz) * (cosf_(ly) * cosf_(lz) + sinf_(lx) * sinf_(ly) * sinf_(lz)) +
                       cosf_(lx) * cosf_(cx) * cosf_(cz) * sinf_(lz);
        float crzcrx = cosf_(lx) * cosf_(lz) * cosf_(cx) * cosf_(cz) -
                       cosf_(cx) * sinf_(cz) * (cosf_(ly) * sinf_(lz) - cosf_(lz) * sinf_(lx) * sinf_(ly)) -
                       sinf_(cx) * (sinf_(ly) * sinf_(lz) + cosf_(ly) * cosf_(lz) * sinf_(lx));
        oz = atan2f_(srzcrx / cosf_(ox), crzcrx / cosf_(ox));
    }

    // ------------------------------------------------------------ correspondences
    static float sq3(const Pt& a, const Pt& b) {  // (ax-bx)^2 + (ay-by)^2 + (az-bz)^2 left to right
        return (a.x - b.x) * (a.x - b.x) + (a.y - b.y) * (a.y - b.y) + (a.z - b.z) * (a.z - b.z);
    }

    void findCorrespondingCornerFeatures(int iterCount) {
        int cornerPointsSharpNum = (int)cornerPointsSharp.size();
        const int lastN = (int)laserCloudCornerLast.size();
        for (int i = 0; i < cornerPointsSharpNum; i++) {
            Pt pointSel;
            TransformToStart(cornerPointsSharp[i], pointSel);
            if (iterCount % 5 == 0) {
                int ni = -1; float nd = FLT_MAX;
                if (kdtreeCornerLast.knn(pointSel, 1, &ni, &nd) == 0 || ni >= lastN) nd = FLT_MAX;
                int closestPointInd = -1, minPointInd2 = -1;
                if (nd < cfg.nearest_feature_search_sq_dist) {
                    closestPointInd = ni;
                    int closestPointScan = (int)laserCloudCornerLast[closestPointInd].intensity;
                    float pointSqDis, minPointSqDis2 = cfg.nearest_feature_search_sq_dist;
                    // Q7: bounded by the current sharp count (and, for memory
                    // safety here, by the previous cloud's size)
                    for (int j = closestPointInd + 1; j < cornerPointsSharpNum && j < lastN; j++) {
                        if ((int)laserCloudCornerLast[j].intensity > closestPointScan + 2.5) break;
                        pointSqDis = sq3(laserCloudCornerLast[j], pointSel);
                        if ((int)laserCloudCornerLast[j].intensity > closestPointScan) {
                            if (pointSqDis < minPointSqDis2) { minPointSqDis2 = pointSqDis; minPointInd2 = j; }
                        }
                    }
                    for (int j = closestPointInd - 1; j >= 0; j--) {
                        if ((int)laserCloudCornerLast[j].intensity < closestPointScan - 2.5) break;
                        pointSqDis = sq3(laserCloudCornerLast[j], pointSel);
                        if ((int)laserCloudCornerLast[j].intensity < closestPointScan) {
                            if (pointSqDis < minPointSqDis2) { minPointSqDis2 = pointSqDis; minPointInd2 = j; }
                        }
                    }
                }
                pointSearchCornerInd1[i] = (float)closestPointInd;
                pointSearchCornerInd2[i] = (float)minPointInd2;
            }
            if (pointSearchCornerInd2[i] >= 0) {
                const Pt& tripod1 = laserCloudCornerLast[(int)pointSearchCornerInd1[i]];
                const Pt& tripod2 = laserCloudCornerLast[(int)pointSearchCornerInd2[i]];
                float x0 = pointSel.x, y0 = pointSel.y, z0 = pointSel.z;
                float x1 = tripod1.x, y1 = tripod1.y, z1 = tripod1.z;
                float x2 = tripod2.x, y2 = tripod2.y, z2 = tripod2.z;
                float m11 = ((x0 - x1) * (y0 - y2) - (x0 - x2) * (y0 - y1));
                float m22 = ((x0 - x1) * (z0 - z2) - (x0 - x2) * (z0 - z1));
                float m33 = ((y0 - y1) * (z0 - z2) - (y0 - y2) * (z0 - z1));
                float a012 = sqrtf(m11 * m11 + m22 * m22 + m33 * m33);
                float l12 = sqrtf((x1 - x2) * (x1 - x2) + (y1 - y2) * (y1 - y2) + (z1 - z2) * (z1 - z2));
                float la = ((y1 - y2) * m11 + (z1 - z2) * m22) / a012 / l12;
                float lb = -((x1 - x2) * m11 - (z1 - z2) * m33) / a012 / l12;
                float lc = -((x1 - x2) * m22 + (y1 - y2) * m33) / a012 / l12;
                float ld2 = a012 / l12;
                float s = 1;
                if (iterCount >= 5) s = (float)(1 - 1.8 * fabsf(ld2));
                if (s > 0.1 && ld2 != 0) {
                    laserCloudOri.push_back(cornerPointsSharp[i]);
                    coeffSel.push_back({s * la, s * lb, s * lc, s * ld2});
                }
            }
        }
    }

    void findCorrespondingSurfFeatures(int iterCount) {
        int surfPointsFlatNum = (int)surfPointsFlat.size();
        const int lastN = (int)laserCloudSurfLast.size();
        for (int i = 0; i < surfPointsFlatNum; i++) {
            Pt pointSel;
            TransformToStart(surfPointsFlat[i], pointSel);
            if (iterCount % 5 == 0) {
                int ni = -1; float nd = FLT_MAX;
                if (kdtreeSurfLast.knn(pointSel, 1, &ni, &nd) == 0 || ni >= lastN) nd = FLT_MAX;
                int closestPointInd = -1, minPointInd2 = -1, minPointInd3 = -1;
                if (nd < cfg.nearest_feature_search_sq_dist) {
                    closestPointInd = ni;
                    int closestPointScan = (int)laserCloudSurfLast[closestPointInd].intensity;
                    float pointSqDis, minPointSqDis2 = cfg.nearest_feature_search_sq_dist,
                                      minPointSqDis3 = cfg.nearest_feature_search_sq_dist;
                    for (int j = closestPointInd + 1; j < surfPointsFlatNum && j < lastN; j++) {
                        if ((int)laserCloudSurfLast[j].intensity > closestPointScan + 2.5) break;
                        pointSqDis = sq3(laserCloudSurfLast[j], pointSel);
                        if ((int)laserCloudSurfLast[j].intensity <= closestPointScan) {
                            if (pointSqDis < minPointSqDis2) { minPointSqDis2 = pointSqDis; minPointInd2 = j; }
                        } else {
                            if (pointSqDis < minPointSqDis3) { minPointSqDis3 = pointSqDis; minPointInd3 = j; }
                        }
                    }
                    for (int j = closestPointInd - 1; j >= 0; j--) {
                        if ((int)laserCloudSurfLast[j].intensity < closestPointScan - 2.5) break;
                        pointSqDis = sq3(laserCloudSurfLast[j], pointSel);
                        if ((int)laserCloudSurfLast[j].intensity >= closestPointScan) {
                            if (pointSqDis < minPointSqDis2) { minPointSqDis2 = pointSqDis; minPointInd2 = j; }
                        } else {
                            if (pointSqDis < minPointSqDis3) { minPointSqDis3 = pointSqDis; minPointInd3 = j; }
                        }
                    }
                }
                pointSearchSurfInd1[i] = (float)closestPointInd;
                pointSearchSurfInd2[i] = (float)minPointInd2;
                pointSearchSurfInd3[i] = (float)minPointInd3;
            }
            if (pointSearchSurfInd2[i] >= 0 && pointSearchSurfInd3[i] >= 0) {
                const Pt& tripod1 = laserCloudSurfLast[(int)pointSearchSurfInd1[i]];
                const Pt& tripod2 = laserCloudSurfLast[(int)pointSearchSurfInd2[i]];
                const Pt& tripod3 = laserCloudSurfLast[(int)pointSearchSurfInd3[i]];
                float pa = (tripod2.y - tripod1.y) * (tripod3.z - tripod1.z) - (tripod3.y - tripod1.y) * (tripod2.z - tripod1.z);
                float pb = (tripod2.z - tripod1.z) * (tripod3.x - tripod1.x) - (tripod3.z - tripod1.z) * (tripod2.x - tripod1.x);
                float pc = (tripod2.x - tripod1.x) * (tripod3.y - tripod1.y) - (tripod3.x - tripod1.x) * (tripod2.y - tripod1.y);
                float pd = -(pa * tripod1.x + pb * tripod1.y + pc * tripod1.z);
                float ps = sqrtf(pa * pa + pb * pb + pc * pc);
                pa /= ps; pb /= ps; pc /= ps; pd /= ps;
                float pd2 = pa * pointSel.x + pb * pointSel.y + pc * pointSel.z + pd;
                float s = 1;
                if (iterCount >= 5)
                    s = (float)(1 - 1.8 * fabsf(pd2) /
                                        sqrtf(sqrtf(pointSel.x * pointSel.x + pointSel.y * pointSel.y + pointSel.z * pointSel.z)));
                if (s > 0.1 && pd2 != 0) {
                    laserCloudOri.push_back(surfPointsFlat[i]);
                    coeffSel.push_back({s * pa, s * pb, s * pc, s * pd2});
                }
            }
        }
    }

    // shared tail of the two 3-DOF solvers (FA:1324-1356 / 1425-1457)
    void solve3(const std::vector<float>& A, const std::vector<float>& B, int n, int iterCount, float* X) {
        float AtA[9], AtB[3];
        gemm_AtA(A, n, 3, AtA);
        gemm_AtB(A, B, n, 3, AtB);
        cv_solve_qr(AtA, AtB, 3, 3, X);
        if (iterCount == 0) {
            float E[3], V[9], V2[9], Vi[9];
            cv_eigen_sym(AtA, 3, E, V);
            memcpy(V2, V, sizeof(V));
            isDegenerate = false;
            const float eignThre[3] = {10, 10, 10};
            for (int i = 2; i >= 0; i--) {
                if (E[i] < eignThre[i]) {
                    for (int j = 0; j < 3; j++) V2[i * 3 + j] = 0;
                    isDegenerate = true;
                } else break;
            }
            cv_inv(V, 3, Vi);
            gemm_small(Vi, V2, 3, 3, 3, matP);
        }
        if (isDegenerate) {
            float X2[3] = {X[0], X[1], X[2]};
            gemm_small(matP, X2, 3, 3, 1, X);
        }
    }

    bool calculateTransformationSurf(int iterCount) {
        using namespace oracle_libm;
        int pointSelNum = (int)laserCloudOri.size();
        std::vector<float> A(pointSelNum * 3), B(pointSelNum);
        float srx = sinf_(transformCur[0]), crx = cosf_(transformCur[0]);
        float sry = sinf_(transformCur[1]), cry = cosf_(transformCur[1]);
        float srz = sinf_(transformCur[2]), crz = cosf_(transformCur[2]);
        float tx = transformCur[3], ty = transformCur[4], tz = transformCur[5];
        float a1 = crx * sry * srz; float a2 = crx * crz * sry; float a3 = srx * sry; float a4 = tx * a1 - ty * a2 - tz * a3;
        float a5 = srx * srz; float a6 = crz * srx; float a7 = ty * a6 - tz * crx - tx * a5;
        float a8 = crx * cry * srz; float a9 = crx * cry * crz; float a10 = cry * srx; float a11 = tz * a10 + ty * a9 - tx * a8;
        float b1 = -crz * sry - cry * srx * srz; float b2 = cry * crz * srx - sry * srz;
        float b5 = cry * crz - srx * sry * srz; float b6 = cry * srz + crz * srx * sry;
        float c1 = -b6; float c2 = b5; float c3 = tx * b6 - ty * b5; float c4 = -crx * crz; float c5 = crx * srz; float c6 = ty * c5 + tx * -c4;
        float c7 = b2; float c8 = -b1; float c9 = tx * -b2 - ty * -b1;
        for (int i = 0; i < pointSelNum; i++) {
            const Pt& p = laserCloudOri[i];
            const Pt& cf = coeffSel[i];
            float arx = (-a1 * p.x + a2 * p.y + a3 * p.z + a4) * cf.x + (a5 * p.x - a6 * p.y + crx * p.z + a7) * cf.y +
                        (a8 * p.x - a9 * p.y - a10 * p.z + a11) * cf.z;
            float arz = (c1 * p.x + c2 * p.y + c3) * cf.x + (c4 * p.x - c5 * p.y + c6) * cf.y + (c7 * p.x + c8 * p.y + c9) * cf.z;
            float aty = -b6 * cf.x + c4 * cf.y + b2 * cf.z;
            A[i * 3 + 0] = arx; A[i * 3 + 1] = arz; A[i * 3 + 2] = aty;
            B[i] = (float)(-0.05 * cf.intensity);
        }
        float X[3];
        solve3(A, B, pointSelNum, iterCount, X);
        transformCur[0] += X[0];
        transformCur[2] += X[1];
        transformCur[4] += X[2];
        for (int i = 0; i < 6; i++) if (std::isnan(transformCur[i])) transformCur[i] = 0;
        double r0 = X[0] * 180.0 / M_PI, r1 = X[1] * 180.0 / M_PI;
        double t2 = (double)(X[2] * 100);
        float deltaR = (float)sqrt(r0 * r0 + r1 * r1);
        float deltaT = (float)sqrt(t2 * t2);
        if (deltaR < 0.1 && deltaT < 0.1) return false;
        return true;
    }

    bool calculateTransformationCorner(int iterCount) {
        using namespace oracle_libm;
        int pointSelNum = (int)laserCloudOri.size();
        std::vector<float> A(pointSelNum * 3), B(pointSelNum);
        float srx = sinf_(transformCur[0]), crx = cosf_(transformCur[0]);
        float sry = sinf_(transformCur[1]), cry = cosf_(transformCur[1]);
        float srz = sinf_(transformCur[2]), crz = cosf_(transformCur[2]);
        float tx = transformCur[3], ty = transformCur[4], tz = transformCur[5];
        float b1 = -crz * sry - cry * srx * srz; float b2 = cry * crz * srx - sry * srz; float b3 = crx * cry; float b4 = tx * -b1 + ty * -b2 + tz * b3;
        float b5 = cry * crz - srx * sry * srz; float b6 = cry * srz + crz * srx * sry; float b7 = crx * sry; float b8 = tz * b7 - ty * b6 - tx * b5;
        float c5 = crx * srz;
        for (int i = 0; i < pointSelNum; i++) {
            const Pt& p = laserCloudOri[i];
            const Pt& cf = coeffSel[i];
            float ary = (b1 * p.x + b2 * p.y - b3 * p.z + b4) * cf.x + (b5 * p.x + b6 * p.y - b7 * p.z + b8) * cf.z;
            float atx = -b5 * cf.x + c5 * cf.y + b1 * cf.z;
            float atz = b7 * cf.x - srx * cf.y - b3 * cf.z;
            A[i * 3 + 0] = ary; A[i * 3 + 1] = atx; A[i * 3 + 2] = atz;
            B[i] = (float)(-0.05 * cf.intensity);
        }
        float X[3];
        solve3(A, B, pointSelNum, iterCount, X);
        transformCur[1] += X[0];
        transformCur[3] += X[1];
        transformCur[5] += X[2];
        for (int i = 0; i < 6; i++) if (std::isnan(transformCur[i])) transformCur[i] = 0;
        double r0 = X[0] * 180.0 / M_PI;
        double t1 = (double)(X[1] * 100), t2 = (double)(X[2] * 100);
        float deltaR = (float)sqrt(r0 * r0);
        float deltaT = (float)sqrt(t1 * t1 + t2 * t2);
        if (deltaR < 0.1 && deltaT < 0.1) return false;
        return true;
    }

    void updateTransformation() {
        iters_surf = iters_corner = 0;
        if (laserCloudCornerLastNum < 10 || laserCloudSurfLastNum < 100) return;
        for (int iterCount1 = 0; iterCount1 < 25; iterCount1++) {
            laserCloudOri.clear(); coeffSel.clear();
            findCorrespondingSurfFeatures(iterCount1);
            iters_surf = iterCount1 + 1;
            if (laserCloudOri.size() < 10) continue;
            if (!calculateTransformationSurf(iterCount1)) break;
        }
        for (int iterCount2 = 0; iterCount2 < 25; iterCount2++) {
            laserCloudOri.clear(); coeffSel.clear();
            findCorrespondingCornerFeatures(iterCount2);
            iters_corner = iterCount2 + 1;
            if (laserCloudOri.size() < 10) continue;
            if (!calculateTransformationCorner(iterCount2)) break;
        }
    }

    void integrateTransformation() {
        using namespace oracle_libm;
        float rx, ry, rz, tx, ty, tz;
        AccumulateRotation(transformSum[0], transformSum[1], transformSum[2], -transformCur[0], -transformCur[1],
                           -transformCur[2], rx, ry, rz);
        float x1 = cosf_(rz) * (transformCur[3] - imuShiftFromStartX) - sinf_(rz) * (transformCur[4] - imuShiftFromStartY);
        float y1 = sinf_(rz) * (transformCur[3] - imuShiftFromStartX) + cosf_(rz) * (transformCur[4] - imuShiftFromStartY);
        float z1 = transformCur[5] - imuShiftFromStartZ;
        float x2 = x1;
        float y2 = cosf_(rx) * y1 - sinf_(rx) * z1;
        float z2 = sinf_(rx) * y1 + cosf_(rx) * z1;
        tx = transformSum[3] - (cosf_(ry) * x2 + sinf_(ry) * z2);
        ty = transformSum[4] - y2;
        tz = transformSum[5] - (-sinf_(ry) * x2 + cosf_(ry) * z2);
        PluginIMURotation(rx, ry, rz, imuPitchStart, imuYawStart, imuRollStart, imuPitchLast, imuYawLast,
                          imuRollLast, rx, ry, rz);
        transformSum[0] = rx; transformSum[1] = ry; transformSum[2] = rz;
        transformSum[3] = tx; transformSum[4] = ty; transformSum[5] = tz;
    }

    void publishCloudsLast() {
        updateImuRollPitchYawStartSinCos();
        for (auto& p : cornerPointsLessSharp) TransformToEnd(p, p);
        for (auto& p : surfPointsLessFlat) TransformToEnd(p, p);
        std::swap(cornerPointsLessSharp, laserCloudCornerLast);
        std::swap(surfPointsLessFlat, laserCloudSurfLast);
        laserCloudCornerLastNum = (int)laserCloudCornerLast.size();
        laserCloudSurfLastNum = (int)laserCloudSurfLast.size();
        if (laserCloudCornerLastNum > 10 && laserCloudSurfLastNum > 100) {
            kdtreeCornerLast.build(laserCloudCornerLast);
            kdtreeSurfLast.build(laserCloudSurfLast);
        }
        frameCount++;
        published_to_mapping = false;
        if (frameCount >= cfg.skip_frame_num + 1) {
            frameCount = 0;
            for (auto& p : outlierCloud) { Pt q{p.y, p.z, p.x, p.intensity}; p = q; }  // adjustOutlierCloud
            published_to_mapping = true;
        }
    }

    void checkSystemInitialization() {
        std::swap(cornerPointsLessSharp, laserCloudCornerLast);
        std::swap(surfPointsLessFlat, laserCloudSurfLast);
        kdtreeCornerLast.build(laserCloudCornerLast);
        kdtreeSurfLast.build(laserCloudSurfLast);
        laserCloudCornerLastNum = (int)laserCloudCornerLast.size();
        laserCloudSurfLastNum = (int)laserCloudSurfLast.size();
        transformSum[0] += imuPitchStart;
        transformSum[2] += imuRollStart;
        systemInitedLM = true;
    }

    void updateInitialGuess() {
        imuPitchLast = imuPitchCur;
        imuYawLast = imuYawCur;
        imuRollLast = imuRollCur;
        imuShiftFromStartX = imuShiftFromStartXCur;
        imuShiftFromStartY = imuShiftFromStartYCur;
        imuShiftFromStartZ = imuShiftFromStartZCur;
        imuVeloFromStartX = imuVeloFromStartXCur;
        imuVeloFromStartY = imuVeloFromStartYCur;
        imuVeloFromStartZ = imuVeloFromStartZCur;
        if (imuAngularFromStartX != 0 || imuAngularFromStartY != 0 || imuAngularFromStartZ != 0) {
            transformCur[0] = -imuAngularFromStartY;
            transformCur[1] = -imuAngularFromStartZ;
            transformCur[2] = -imuAngularFromStartX;
        }
        if (imuVeloFromStartX != 0 || imuVeloFromStartY != 0 || imuVeloFromStartZ != 0) {
            transformCur[3] -= imuVeloFromStartX * cfg.scan_period;
            transformCur[4] -= imuVeloFromStartY * cfg.scan_period;
            transformCur[5] -= imuVeloFromStartZ * cfg.scan_period;
        }
    }

    // runFeatureAssociation (FA:1817-1860) on one segmented scan stamped t
    // (cloudHeader.stamp: read only by the IMU path)
    void run(const Cloud& seg, const SegInfo& info, const Cloud& outlier, double t) {
        timeScanCur = t;
        segmentedCloud = seg;
        segInfo = info;
        outlierCloud = outlier;
        published_to_mapping = false;
        adjustDistortion();
        calculateSmoothness();
        markOccludedPoints();
        extractFeatures();
        if (!systemInitedLM) {
            checkSystemInitialization();
            return;
        }
        updateInitialGuess();
        updateTransformation();
        integrateTransformation();
        publishCloudsLast();
    }
};

}  // namespace oracle
