// slo_gendev.hip — the synthetic stream generator (slo_gen.h) on the device.
//
// Benchmark inputs only: the reference ships no data, so every
// scan comes from slo_gen's deterministic city loop.  The host generator costs
// ~1.4 ms per 64x1800 scan per core; a steady-state run of hundreds of
// streams needs 10^5 scans, so generation moves to the GPU.  The host keeps
// the parts that need libm trig or irregular control flow — ray direction
// tables, the pose of every scan (path_at) with its yaw cos/sin, and the
// objects in range of that pose (cull) — and the device evaluates
// slo_gen::ray_point, the same source the host loop runs, so the output is
// bit-identical to slo_gen_batch (tests/test_gpu_gen.py).
//
// Launch: one workgroup per (job = scan x stream, block of 256 rays); the
// job's culled boxes and poles are staged in LDS once per workgroup; every
// thread traces one ray and writes one float4 (coalesced: consecutive rays
// are consecutive points of the firing order).
#include "slo_internal.h"
#include "../../include/slo_abi.h"
#include "slo_gen.h"

#include <string.h>
#include <new>
#include <vector>

namespace {

struct GenJob {
    double px, py, pz, cyaw, syaw;
    uint64_t scene_seed, scan_seed;
    int box_off, nbox, pole_off, npole;
};

constexpr int kGenBlock = 256;

__global__ void __launch_bounds__(kGenBlock) k_gen_scan(const GenJob* __restrict__ jobs,
                                                        const slo_gen::Box* __restrict__ boxes,
                                                        const slo_gen::Pole* __restrict__ poles,
                                                        const double* __restrict__ rays,  // ce[R] se[R] ca[C] sa[C]
                                                        int R, int C, int max_points, float4* __restrict__ out) {
    extern __shared__ char lds[];
    const GenJob J = jobs[blockIdx.y];
    slo_gen::Box* sb = (slo_gen::Box*)lds;
    slo_gen::Pole* sp = (slo_gen::Pole*)(lds + sizeof(slo_gen::Box) * J.nbox);
    for (int b = threadIdx.x; b < J.nbox; b += blockDim.x) sb[b] = boxes[J.box_off + b];
    for (int p = threadIdx.x; p < J.npole; p += blockDim.x) sp[p] = poles[J.pole_off + p];
    __syncthreads();
    const int n = blockIdx.x * kGenBlock + threadIdx.x;
    if (n >= R * C) return;
    const int f = n / R, i = n - f * R;
    float o[4];
    slo_gen::ray_point(rays[2 * R + f], rays[2 * R + C + f], rays[i], rays[R + i], J.px, J.py, J.pz, J.cyaw, J.syaw,
                       sb, J.nbox, sp, J.npole, J.scene_seed, J.scan_seed, (uint64_t)n, o);
    out[(size_t)blockIdx.y * max_points + n] = make_float4(o[0], o[1], o[2], o[3]);
}

}  // namespace

struct slo_gen_dev {
    slo_config cfg;
    int dev = 0;
    int config_id = 0, stream0 = 0, n_streams = 0;
    std::vector<slo_gen::Stream> streams;
    double* d_rays = nullptr;
    // per-call staging (grown on demand)
    GenJob* d_jobs = nullptr;
    slo_gen::Box* d_boxes = nullptr;
    slo_gen::Pole* d_poles = nullptr;
    size_t cap_jobs = 0, cap_boxes = 0, cap_poles = 0;
};

namespace {

template <class T>
int grow(T** p, size_t* cap, size_t want) {
    if (want <= *cap) return SLO_OK;
    if (*p) hipFree(*p);
    *p = nullptr;
    size_t n = want + want / 2 + 16;
    if (hipMalloc((void**)p, n * sizeof(T)) != hipSuccess) { *cap = 0; return SLO_E_HIP; }
    *cap = n;
    return SLO_OK;
}

}  // namespace

extern "C" {

int slo_gen_device_create(int preset, int config_id, int stream0, int n_streams, int hip_device, slo_gen_dev** out) {
    if (!out || n_streams <= 0) return SLO_E_ARG;
    *out = nullptr;
    slo_gen_dev* g = new (std::nothrow) slo_gen_dev();
    if (!g) return SLO_E_CAPACITY;
    if (slo_config_preset_impl(preset, &g->cfg)) { delete g; return SLO_E_ARG; }
    g->dev = hip_device;
    g->config_id = config_id;
    g->stream0 = stream0;
    g->n_streams = n_streams;
    for (int s = 0; s < n_streams; ++s) g->streams.push_back(slo_gen::make_stream(g->cfg, config_id, stream0 + s));
    const int R = g->cfg.n_scan, C = g->cfg.horizon_scan;
    const slo_gen::RayTables& rt = g->streams[0].rays;   // a function of the sensor preset only
    std::vector<double> rays;
    rays.insert(rays.end(), rt.ce.begin(), rt.ce.end());
    rays.insert(rays.end(), rt.se.begin(), rt.se.end());
    rays.insert(rays.end(), rt.ca.begin(), rt.ca.end());
    rays.insert(rays.end(), rt.sa.begin(), rt.sa.end());
    if (hipSetDevice(hip_device) != hipSuccess || hipMalloc((void**)&g->d_rays, rays.size() * 8) != hipSuccess ||
        hipMemcpy(g->d_rays, rays.data(), rays.size() * 8, hipMemcpyHostToDevice) != hipSuccess) {
        slo_gen_device_destroy(g);
        return SLO_E_HIP;
    }
    (void)R; (void)C;
    *out = g;
    return SLO_OK;
}

void slo_gen_device_destroy(slo_gen_dev* g) {
    if (!g) return;
    hipSetDevice(g->dev);
    hipFree(g->d_rays);
    hipFree(g->d_jobs);
    hipFree(g->d_boxes);
    hipFree(g->d_poles);
    delete g;
}

int slo_gen_device_scans(slo_gen_dev* g, int scan0, int n_scans, void* d_out, void* hip_stream) {
    if (!g || !d_out || n_scans <= 0) return SLO_E_ARG;
    if (hipSetDevice(g->dev) != hipSuccess) return SLO_E_HIP;
    const int R = g->cfg.n_scan, C = g->cfg.horizon_scan, S = g->n_streams;
    std::vector<GenJob> jobs((size_t)n_scans * S);
    std::vector<slo_gen::Box> boxes, bb;
    std::vector<slo_gen::Pole> poles, pp;
    size_t max_lds = 0;
    for (int k = 0; k < n_scans; ++k)
        for (int s = 0; s < S; ++s) {
            const slo_gen::Stream& st = g->streams[s];
            const int scan = scan0 + k;
            // stream_scan: the pose at arc offset + speed * k, scan seed = stream seed + k
            slo_gen::SensorPose p = slo_gen::stream_pose(st.scene, st.offset + st.speed * scan);
            slo_gen::cull(st.scene, p, bb, pp);
            GenJob& J = jobs[(size_t)k * S + s];
            J.px = p.x; J.py = p.y; J.pz = p.z;
            J.cyaw = cos(p.yaw); J.syaw = sin(p.yaw);
            J.scene_seed = st.scene.seed;
            J.scan_seed = st.seed + (uint64_t)scan;
            J.box_off = (int)boxes.size(); J.nbox = (int)bb.size();
            J.pole_off = (int)poles.size(); J.npole = (int)pp.size();
            boxes.insert(boxes.end(), bb.begin(), bb.end());
            poles.insert(poles.end(), pp.begin(), pp.end());
            max_lds = std::max(max_lds, bb.size() * sizeof(slo_gen::Box) + pp.size() * sizeof(slo_gen::Pole));
        }
    if (max_lds > 64 * 1024) return SLO_E_CAPACITY;   // a scene far denser than slo_gen makes
    if (jobs.size() > 65535u) return SLO_E_ARG;        // grid.y limit: callers chunk their scans
    int rc;
    if ((rc = grow(&g->d_jobs, &g->cap_jobs, jobs.size())) || (rc = grow(&g->d_boxes, &g->cap_boxes, boxes.size() + 1)) ||
        (rc = grow(&g->d_poles, &g->cap_poles, poles.size() + 1)))
        return rc;
    hipStream_t st = (hipStream_t)hip_stream;
    // the staging vectors die with this call: synchronous copies, then the launch
    if (hipMemcpy(g->d_jobs, jobs.data(), jobs.size() * sizeof(GenJob), hipMemcpyHostToDevice) != hipSuccess ||
        (!boxes.empty() &&
         hipMemcpy(g->d_boxes, boxes.data(), boxes.size() * sizeof(slo_gen::Box), hipMemcpyHostToDevice) != hipSuccess) ||
        (!poles.empty() &&
         hipMemcpy(g->d_poles, poles.data(), poles.size() * sizeof(slo_gen::Pole), hipMemcpyHostToDevice) != hipSuccess))
        return SLO_E_HIP;
    dim3 grid((R * C + kGenBlock - 1) / kGenBlock, (unsigned)jobs.size());
    hipLaunchKernelGGL(k_gen_scan, grid, dim3(kGenBlock), max_lds, st, g->d_jobs, g->d_boxes, g->d_poles, g->d_rays, R,
                       C, g->cfg.max_points, (float4*)d_out);
    if (hipGetLastError() != hipSuccess) return SLO_E_HIP;
    return hipStreamSynchronize(st) == hipSuccess ? SLO_OK : SLO_E_HIP;
}

}  // extern "C"
