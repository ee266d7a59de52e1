// slo_gen.h — deterministic synthetic LiDAR stream generator (host C++).
//
// The reference ships no data; every benchmark and parity
// case runs on scans from this generator.  A stream is a closed urban loop
// (rounded rectangle, ~400 m) lined with building facades, poles and parked
// cars over a slightly rough ground plane.  The sensor drives the loop at
// `speed` metres per scan (10 Hz), so the stream revisits places and Scan
// Context loop detection fires on the second lap.
//
// Points are emitted in firing order — column-major, per azimuth all rings,
// starting behind the sensor and sweeping clockwise like a Velodyne/Ouster —
// because findStartEndAngle (imageProjection.cpp:199-209) and the deskew latch
// (featureAssociation.cpp:505-520) depend on it.  Every ray yields one point;
// no-return and 3 % random drop-outs are emitted as NaN so that
// removeNaNFromPointCloud (imageProjection.cpp:170) is exercised.
//
// Everything is integer hashing plus +,-,*,/,sqrt and slo_libm trig, so the
// stream is bit-identical on every host.  The per-ray work (ray_point) is
// __host__ __device__: it uses only IEEE-exact operations (+ - * / sqrt
// floor fabs, integer hashing) on values the host prepares once — ray
// direction tables, the sensor pose with its yaw cos/sin, the objects near
// the pose — so the device generator (slo_gendev.hip) emits the same bits
// as the host loop below (tests/test_gpu_gen.py).
#pragma once

#include <stdint.h>
#include <math.h>
#include <vector>
#include <algorithm>
#include "slo_config.h"
#include "slo_libm.h"

#if defined(__HIPCC__)
#include <hip/hip_runtime.h>
#define SLO_GEN_HD __host__ __device__ inline
#else
#define SLO_GEN_HD inline
#endif

namespace slo_gen {

SLO_GEN_HD uint64_t mix64(uint64_t x) {
    x ^= x >> 30; x *= 0xbf58476d1ce4e5b9ULL;
    x ^= x >> 27; x *= 0x94d049bb133111ebULL;
    x ^= x >> 31;
    return x;
}
// uniform in [0,1)
SLO_GEN_HD double u01(uint64_t h) { return (double)(mix64(h) >> 11) * (1.0 / 9007199254740992.0); }
// approx N(0,1) by Irwin-Hall(4): pure arithmetic, platform independent
SLO_GEN_HD double gauss(uint64_t h) {
    double s = u01(h) + u01(h ^ 0x9e3779b97f4a7c15ULL) + u01(h ^ 0x3c6ef372fe94f82bULL) +
               u01(h ^ 0xdaa66d2c7ddf743fULL);
    return (s - 2.0) * 1.7320508075688772;  // var(sum)=1/3
}

struct Box { float x0, y0, z0, x1, y1, z1; };
struct Pole { float cx, cy, r, h; };

struct Scene {
    std::vector<Box> boxes;
    std::vector<Pole> poles;
    float half_w = 100.f, half_h = 60.f, corner_r = 20.f;  // loop shape
    uint64_t seed = 0;
};

// Loop path: rounded rectangle centred on the origin.
struct PathPt { double x, y, heading; };

inline double path_length(const Scene& s) {
    double a = 2.0 * (s.half_w - s.corner_r), b = 2.0 * (s.half_h - s.corner_r);
    return 2.0 * (a + b) + 2.0 * M_PI * s.corner_r;
}

inline PathPt path_at(const Scene& s, double arc) {
    const double a = 2.0 * (s.half_w - s.corner_r), b = 2.0 * (s.half_h - s.corner_r);
    const double q = 0.5 * M_PI * s.corner_r;
    const double L = path_length(s);
    arc = fmod(arc, L);
    if (arc < 0) arc += L;
    const double segs[8] = {a, q, b, q, a, q, b, q};
    // start at bottom-left straight, heading +x
    double x = -(s.half_w - s.corner_r), y = -s.half_h, h = 0.0;
    for (int i = 0; i < 8; ++i) {
        double len = segs[i];
        if (arc <= len || i == 7) {
            if ((i & 1) == 0) {
                return {x + cos(h) * arc, y + sin(h) * arc, h};
            } else {
                double ang = arc / s.corner_r;
                double cx = x - sin(h) * s.corner_r, cy = y + cos(h) * s.corner_r;
                double h2 = h + ang;
                return {cx + sin(h2) * s.corner_r, cy - cos(h2) * s.corner_r, h2};
            }
        }
        arc -= len;
        if ((i & 1) == 0) { x += cos(h) * len; y += sin(h) * len; }
        else {
            double cx = x - sin(h) * s.corner_r, cy = y + cos(h) * s.corner_r;
            h += 0.5 * M_PI;
            x = cx + sin(h) * s.corner_r; y = cy - cos(h) * s.corner_r;
        }
    }
    return {x, y, h};
}

// Procedural city along the loop: facades on both sides of the road with
// gaps, poles every ~12 m, parked cars.  Deterministic in `seed`.
inline Scene make_scene(uint64_t seed) {
    Scene sc;
    sc.seed = seed;
    const double L = path_length(sc);
    uint64_t k = 0;
    for (double arc = 0; arc < L; arc += 6.0 + 10.0 * u01(seed * 7919 + (k++))) {
        PathPt p = path_at(sc, arc);
        double nx = -sin(p.heading), ny = cos(p.heading);
        double tx = cos(p.heading), ty = sin(p.heading);
        for (int side = -1; side <= 1; side += 2) {
            uint64_t h = mix64(seed ^ (k * 131 + (side + 2)));
            if (u01(h) < 0.15) continue;  // gap (side street)
            double off = 9.0 + 6.0 * u01(h + 1);
            double len = 5.0 + 9.0 * u01(h + 2);
            double dep = 6.0 + 8.0 * u01(h + 3);
            double hgt = 8.0 + 22.0 * u01(h + 4);
            double cx = p.x + nx * side * (off + 0.5 * dep), cy = p.y + ny * side * (off + 0.5 * dep);
            // axis-aligned footprint approximating the rotated block
            double ex = 0.5 * (fabs(tx) * len + fabs(nx) * dep);
            double ey = 0.5 * (fabs(ty) * len + fabs(ny) * dep);
            sc.boxes.push_back({(float)(cx - ex), (float)(cy - ey), 0.f, (float)(cx + ex),
                                (float)(cy + ey), (float)hgt});
        }
    }
    k = 0;
    for (double arc = 3.0; arc < L; arc += 12.0, ++k) {
        PathPt p = path_at(sc, arc);
        double nx = -sin(p.heading), ny = cos(p.heading);
        uint64_t h = mix64(seed * 31 + k);
        int side = (h & 1) ? 1 : -1;
        double off = 6.0 + 1.5 * u01(h + 9);
        sc.poles.push_back({(float)(p.x + nx * side * off), (float)(p.y + ny * side * off), 0.15f,
                            (float)(5.0 + 4.0 * u01(h + 10))});
        if (u01(h + 11) < 0.5) {  // parked car
            double cx = p.x + nx * (-side) * 4.5 + cos(p.heading) * 4.0;
            double cy = p.y + ny * (-side) * 4.5 + sin(p.heading) * 4.0;
            double ex = 0.5 * (fabs(cos(p.heading)) * 4.4 + fabs(nx) * 1.8);
            double ey = 0.5 * (fabs(sin(p.heading)) * 4.4 + fabs(ny) * 1.8);
            sc.boxes.push_back({(float)(cx - ex), (float)(cy - ey), 0.f, (float)(cx + ex),
                                (float)(cy + ey), 1.5f});
        }
    }
    return sc;
}

// lattice value of ground_height (the signed products wrap, computed unsigned)
SLO_GEN_HD double ground_lattice(uint64_t seed, int64_t a, int64_t b) {
    return 0.02 * (2.0 * u01((seed * 1000003ULL + (uint64_t)a * 73856093ULL) ^ ((uint64_t)b * 19349663ULL)) - 1.0);
}

SLO_GEN_HD float ground_height_seed(uint64_t seed, double x, double y) {
    // smooth-ish roughness (+-2 cm) from a hashed 2 m lattice, bilinear
    double gx = x * 0.5, gy = y * 0.5;
    double fx = floor(gx), fy = floor(gy);
    int64_t ix = (int64_t)fx, iy = (int64_t)fy;
    double tx = gx - fx, ty = gy - fy;
    double v = (1 - tx) * (1 - ty) * ground_lattice(seed, ix, iy) + tx * (1 - ty) * ground_lattice(seed, ix + 1, iy) +
               (1 - tx) * ty * ground_lattice(seed, ix, iy + 1) + tx * ty * ground_lattice(seed, ix + 1, iy + 1);
    return (float)v;
}

inline float ground_height(const Scene& s, double x, double y) { return ground_height_seed(s.seed, x, y); }

struct SensorPose { double x, y, z, yaw; };

inline SensorPose stream_pose(const Scene& s, double arc) {
    PathPt p = path_at(s, arc);
    return {p.x, p.y, 1.73, p.heading};
}

// Ray tables for a config: elevation per row (ang_bottom, ang_res_y),
// azimuth per firing column.  Column f fires at azimuth pi - (f+0.5)*2pi/C
// (behind the sensor, sweeping clockwise).
struct RayTables {
    std::vector<double> ce, se;   // per row
    std::vector<double> ca, sa;   // per firing column
};

inline RayTables make_rays(const slo_config& cfg) {
    RayTables t;
    const int R = cfg.n_scan, C = cfg.horizon_scan;
    for (int i = 0; i < R; ++i) {
        // centre of row i's bin, small per-ring jitter so rows don't sit on bin edges
        double el = (-(double)cfg.ang_bottom + (i + 0.5) * (double)cfg.ang_res_y) * M_PI / 180.0;
        t.ce.push_back(cos(el));
        t.se.push_back(sin(el));
    }
    for (int f = 0; f < C; ++f) {
        double az = M_PI - (f + 0.37) * 2.0 * M_PI / C;
        t.ca.push_back(cos(az));
        t.sa.push_back(sin(az));
    }
    return t;
}

// One ray: firing column direction (ca, sa) in the sensor frame, ring
// elevation (ce, se), the sensor pose (its yaw cos/sin precomputed), the
// objects near the pose in scene order.  Writes x, y, z, intensity (NaN for
// no return / drop-out).
SLO_GEN_HD void ray_point(double ca, double sa, double ce, double se, double px, double py, double pz,
                          double cyaw, double syaw, const Box* boxes, int nbox, const Pole* poles, int npole,
                          uint64_t scene_seed, uint64_t scan_seed, uint64_t ray_index, float* o) {
    const double maxr = 120.0;
    // world-frame horizontal direction of this firing column
    double dxh = ca * cyaw - sa * syaw;
    double dyh = ca * syaw + sa * cyaw;
    double dx = dxh * ce, dy = dyh * ce, dz = se;
    double tbest = maxr;
    int kind = 0;
    if (dz < -1e-6) {
        double t = (pz - 0.0) / (-dz);
        if (t < tbest) {
            double gx = px + dx * t, gy = py + dy * t;
            double gz = ground_height_seed(scene_seed, gx, gy);
            t = (pz - gz) / (-dz);
            if (t < tbest) { tbest = t; kind = 1; }
        }
    }
    for (int bi = 0; bi < nbox; ++bi) {
        const Box& B = boxes[bi];
        double t0 = 0.0, t1 = tbest;
        const double org[3] = {px, py, pz};
        const double d[3] = {dx, dy, dz};
        const double lo[3] = {B.x0, B.y0, B.z0}, hi[3] = {B.x1, B.y1, B.z1};
        bool hit = true;
        for (int a = 0; a < 3 && hit; ++a) {
            if (fabs(d[a]) < 1e-12) {
                if (org[a] < lo[a] || org[a] > hi[a]) hit = false;
            } else {
                double inv = 1.0 / d[a];
                double ta = (lo[a] - org[a]) * inv, tb = (hi[a] - org[a]) * inv;
                if (ta > tb) { double tmp = ta; ta = tb; tb = tmp; }
                if (ta > t0) t0 = ta;
                if (tb < t1) t1 = tb;
                if (t0 > t1) hit = false;
            }
        }
        if (hit && t0 > 0.5 && t0 < tbest) { tbest = t0; kind = 2; }
    }
    for (int pi = 0; pi < npole; ++pi) {
        const Pole& P = poles[pi];
        double ox = px - P.cx, oy = py - P.cy;
        double a = dx * dx + dy * dy, b = 2 * (ox * dx + oy * dy), c = ox * ox + oy * oy - (double)P.r * P.r;
        double disc = b * b - 4 * a * c;
        if (disc < 0 || a < 1e-12) continue;
        double t = (-b - sqrt(disc)) / (2 * a);
        if (t > 0.5 && t < tbest) {
            double z = pz + dz * t;
            if (z >= 0 && z <= P.h) { tbest = t; kind = 3; }
        }
    }
    uint64_t h = mix64(scan_seed * 0x100000001b3ULL + ray_index);
    if (kind == 0 || u01(h) < 0.03) {
        const float qnan = __builtin_nanf("");
        o[0] = o[1] = o[2] = qnan; o[3] = qnan;
    } else {
        double r = tbest + 0.02 * gauss(h + 17);
        // sensor frame: x forward, y left, z up
        double lx = ca * ce * r, ly = sa * ce * r, lz = se * r;
        o[0] = (float)lx; o[1] = (float)ly; o[2] = (float)lz;
        o[3] = (float)u01(h + 29);
    }
}

// Objects within the sensor's range of `pose`, in scene order (ties in the
// nearest-hit test go to the earlier object, so the order is part of the data)
inline void cull(const Scene& sc, const SensorPose& pose, std::vector<Box>& boxes, std::vector<Pole>& poles) {
    const double maxr = 120.0;
    boxes.clear();
    poles.clear();
    for (int b = 0; b < (int)sc.boxes.size(); ++b) {
        const Box& B = sc.boxes[b];
        double dx = std::max({(double)B.x0 - pose.x, 0.0, pose.x - (double)B.x1});
        double dy = std::max({(double)B.y0 - pose.y, 0.0, pose.y - (double)B.y1});
        if (dx * dx + dy * dy < maxr * maxr) boxes.push_back(B);
    }
    for (int p = 0; p < (int)sc.poles.size(); ++p) {
        double dx = sc.poles[p].cx - pose.x, dy = sc.poles[p].cy - pose.y;
        if (dx * dx + dy * dy < maxr * maxr) poles.push_back(sc.poles[p]);
    }
}

// Generate one scan into out (x,y,z,intensity) float4s, R*C points.
// Returns the number of points written (= R*C; NaN for no return).
inline int generate_scan(const slo_config& cfg, const Scene& sc, const RayTables& rt,
                         const SensorPose& pose, uint64_t scan_seed, float* out) {
    const int R = cfg.n_scan, C = cfg.horizon_scan;
    const double cyaw = cos(pose.yaw), syaw = sin(pose.yaw);
    std::vector<Box> boxes;
    std::vector<Pole> poles;
    cull(sc, pose, boxes, poles);
    int n = 0;
    for (int f = 0; f < C; ++f)
        for (int i = 0; i < R; ++i) {
            ray_point(rt.ca[f], rt.sa[f], rt.ce[i], rt.se[i], pose.x, pose.y, pose.z, cyaw, syaw, boxes.data(),
                      (int)boxes.size(), poles.data(), (int)poles.size(), sc.seed, scan_seed,
                      (uint64_t)(f * R + i), out + 4 * (size_t)n);
            ++n;
        }
    return n;
}

// A stream = scene + start offset; scan k is at arc = offset + speed*k.
struct Stream {
    slo_config cfg;
    Scene scene;
    RayTables rays;
    double offset = 0, speed = 1.0;
    uint64_t seed = 0;
};

inline Stream make_stream(const slo_config& cfg, int config_id, int stream_id, double speed = 1.0) {
    Stream s;
    s.cfg = cfg;
    s.seed = 0x5C1E60ULL + (uint64_t)config_id * 1000003ULL + (uint64_t)stream_id * 7777777ULL;
    s.scene = make_scene(s.seed);
    s.rays = make_rays(cfg);
    s.offset = 37.0 * stream_id;
    s.speed = speed;
    return s;
}

inline int stream_scan(const Stream& s, int k, float* out) {
    SensorPose p = stream_pose(s.scene, s.offset + s.speed * k);
    return generate_scan(s.cfg, s.scene, s.rays, p, s.seed + (uint64_t)k, out);
}

}  // namespace slo_gen
