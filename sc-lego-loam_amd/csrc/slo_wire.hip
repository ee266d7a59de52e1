// slo_wire.hip — sensor_msgs/PointCloud2 ingestion.
//
// ImageProjection::copyPointCloud (imageProjection.cpp:165-170) converts the
// message with pcl::fromROSMsg into pcl::PointCloud<PointXYZI> before
// projecting.  fromROSMsg (pcl_conversions) hands the message to
// pcl::fromPCLPointCloud2 (pcl/conversions.h), whose rules this file keeps:
//   * createMapping: for every field of the point type (x, y, z, intensity,
//     all float) the FIRST message field with the same name, datatype FLOAT32
//     and count 1 (or 0: a count of 0 is accepted for scalar fields) is used;
//     a point-type field with no match is left as constructed (PointXYZI()
//     zeroes x, y, z, intensity) and PCL only warns;
//   * copy: point (row, col) is read at data + row * row_step + col *
//     point_step, field bytes copied as they are (is_bigendian is not looked
//     at);
//   * width * height points come out, NaNs included — removeNaNFromPointCloud
//     (IP:170) runs inside the projection kernel, not here.
// The single-scan path converts on the host (the reference's own callback
// owns one message); the batched path uploads the raw message bytes and
// unpacks them on the device, one thread per point, so a batch of messages
// costs one HBM pass instead of a host loop per stream.
#include <hip/hip_runtime.h>
#include <string.h>
#include <cmath>
#include <vector>
#include "slo_internal.h"

namespace {

// FieldMatches<PointT, Tag> for a scalar float field (pcl/conversions.h)
int match_field(const slo_pc2* m, const char* name, int datatype = SLO_PF_FLOAT32) {
    for (int k = 0; k < m->n_fields; ++k) {
        const slo_pc2_field& f = m->fields[k];
        if (!f.name || strcmp(f.name, name) != 0) continue;
        if (f.datatype == datatype && (f.count == 1 || f.count == 0)) return (int)f.offset;
    }
    return -1;
}

int layout_of(const slo_pc2* m, slo_pc2_layout* L) {
    if (!m || !L || (m->n_fields > 0 && !m->fields) || m->n_fields < 0) return SLO_E_ARG;
    L->point_step = m->point_step;
    L->off_x = match_field(m, "x");
    L->off_y = match_field(m, "y");
    L->off_z = match_field(m, "z");
    L->off_intensity = match_field(m, "intensity");
    L->off_ring = match_field(m, "ring", SLO_PF_UINT16);   // PointXYZIR's uint16 ring (utility.h:158-169)
    for (int o : {L->off_x, L->off_y, L->off_z, L->off_intensity})
        if (o >= 0 && (uint64_t)o + 4 > m->point_step) return SLO_E_ARG;
    if (L->off_ring >= 0 && (uint64_t)L->off_ring + 2 > m->point_step) return SLO_E_ARG;
    return SLO_OK;
}

inline float read_f32(const uint8_t* p, int off) {
    float v = 0.0f;
    if (off >= 0) memcpy(&v, p + off, 4);
    return v;
}

// last byte the message's points touch (0 for an empty cloud)
uint64_t bytes_needed(const slo_pc2* m) {
    if (!m->width || !m->height) return 0;
    return (uint64_t)(m->height - 1) * m->row_step + (uint64_t)(m->width - 1) * m->point_step + m->point_step;
}

int to_xyzi(const slo_pc2* m, float* out, size_t cap, size_t* n_out) {
    slo_pc2_layout L;
    int r = layout_of(m, &L);
    if (r) return r;
    if (!n_out) return SLO_E_ARG;
    const size_t n = (size_t)m->width * m->height;
    *n_out = n;
    if (n && (!m->data || !out)) return SLO_E_ARG;
    if (bytes_needed(m) > m->data_bytes) return SLO_E_ARG;
    if (n > cap) return SLO_E_CAPACITY;
    size_t i = 0;
    for (uint32_t row = 0; row < m->height; ++row) {
        const uint8_t* rp = m->data + (size_t)row * m->row_step;
        for (uint32_t col = 0; col < m->width; ++col, ++i) {
            const uint8_t* p = rp + (size_t)col * m->point_step;
            out[4 * i] = read_f32(p, L.off_x);
            out[4 * i + 1] = read_f32(p, L.off_y);
            out[4 * i + 2] = read_f32(p, L.off_z);
            out[4 * i + 3] = read_f32(p, L.off_intensity);
        }
    }
    return SLO_OK;
}

// one thread per point; blockIdx.y = stream.  The four field reads are dword
// loads when the layout and the message's row_step are 4-byte aligned (every
// LiDAR driver's are), byte loads otherwise (uniform per workgroup).
__global__ void __launch_bounds__(256) k_pc2_unpack(const uint8_t* __restrict__ bytes, size_t msg_stride,
                                                    const int32_t* __restrict__ dims, slo_pc2_layout L, int P,
                                                    bool layout_aligned, float4* __restrict__ out,
                                                    int32_t* __restrict__ counts, uint16_t* __restrict__ rings,
                                                    slo::StreamState* st) {
    const int s = blockIdx.y;
    const int w = dims[3 * s], h = dims[3 * s + 1], row_step = dims[3 * s + 2];
    long long n_all = (long long)max(w, 0) * max(h, 0);
    // a message whose points would reach past its slot (or a negative
    // row_step) is not read at all: count 0 and the input error bit
    const bool fits = n_all == 0 || (row_step >= 0 && (long long)(h - 1) * row_step +
                                     (long long)(w - 1) * L.point_step + L.point_step <= (long long)msg_stride);
    if (!fits) n_all = 0;
    const int n = (int)min(n_all, (long long)P);
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i == 0) {
        counts[s] = n;
        if (n_all > P || !fits) atomicOr(&st[s].err, SLO_ERR_INPUT);
    }
    if (i >= n) return;
    const bool aligned = layout_aligned && (row_step & 3) == 0;
    const int row = i / w, col = i - row * w;
    const uint8_t* p = bytes + (size_t)s * msg_stride + (size_t)row * row_step + (size_t)col * L.point_step;
    auto rd = [&](int off) -> float {
        if (off < 0) return 0.0f;
        if (aligned) return *(const float*)(p + off);
        const unsigned int u = (unsigned int)p[off] | ((unsigned int)p[off + 1] << 8) |
                               ((unsigned int)p[off + 2] << 16) | ((unsigned int)p[off + 3] << 24);
        return __uint_as_float(u);
    };
    out[(size_t)s * P + i] = make_float4(rd(L.off_x), rd(L.off_y), rd(L.off_z), rd(L.off_intensity));
    if (rings) {
        const int o = L.off_ring;
        rings[(size_t)s * P + i] = o < 0 ? 0 : (uint16_t)(p[o] | (p[o + 1] << 8));
    }
}

}  // namespace

extern "C" {

int slo_pc2_layout_of(const slo_pc2* msg, slo_pc2_layout* out) { return layout_of(msg, out); }

int slo_pc2_to_xyzi(const slo_pc2* msg, float* out_xyzi, size_t cap_points, size_t* n_out) {
    return to_xyzi(msg, out_xyzi, cap_points, n_out);
}

int slo_image_projection_pc2(slo_ctx* ctx, const slo_pc2* msg, slo_seg_view* out) {
    if (!ctx || !msg || !out) return SLO_E_ARG;
    thread_local std::vector<float> buf;
    thread_local std::vector<uint16_t> ring_raw, ring_eff;
    const size_t n = (size_t)msg->width * msg->height;
    if (n > (size_t)ctx->cfg.max_points) { ctx->err = "too many points"; return SLO_E_CAPACITY; }
    buf.resize(4 * std::max<size_t>(n, 1));
    size_t got = 0;
    const int r = to_xyzi(msg, buf.data(), n, &got);
    if (r) { ctx->err = "malformed PointCloud2"; return r; }
    if (!ctx->cfg.use_cloud_ring) return slo_image_projection(ctx, buf.data(), got, 16, 0, 12, out);
    // useCloudRing (IP:172-178): fromROSMsg into PointXYZIR, whose is_dense
    // must be set (else the reference shuts down), then row = the ring of
    // laserCloudInRing->points[i] with i the index after NaN removal
    if (!msg->is_dense) { ctx->err = "useCloudRing needs an is_dense cloud (IP:174-177)"; return SLO_E_ARG; }
    slo_pc2_layout L;
    layout_of(msg, &L);
    ring_raw.assign(std::max<size_t>(n, 1), 0);
    ring_eff.assign(std::max<size_t>(n, 1), 0);
    size_t i = 0;
    for (uint32_t row = 0; row < msg->height; ++row)
        for (uint32_t col = 0; col < msg->width; ++col, ++i)
            if (L.off_ring >= 0)
                memcpy(&ring_raw[i], msg->data + (size_t)row * msg->row_step + (size_t)col * msg->point_step + L.off_ring, 2);
    size_t f = 0;   // filtered index of each finite point
    for (size_t k = 0; k < n; ++k) {
        const float* p = &buf[4 * k];
        if (std::isfinite(p[0]) && std::isfinite(p[1]) && std::isfinite(p[2])) ring_eff[k] = ring_raw[f++];
    }
    return slo_image_projection_ring(ctx, buf.data(), got, 16, 0, 12, ring_eff.data(), out);
}

int slo_batch_pc2_unpack(slo_ctx* ctx, const uint8_t* d_bytes, size_t msg_stride, const int32_t* d_dims,
                         const slo_pc2_layout* layout, void* d_points, int32_t* d_counts, uint16_t* d_rings) {
    if (!ctx || !d_bytes || !d_dims || !layout || !d_points || !d_counts) return SLO_E_ARG;
    const slo_pc2_layout L = *layout;
    for (int o : {L.off_x, L.off_y, L.off_z, L.off_intensity})
        if (o >= 0 && (uint64_t)o + 4 > L.point_step) { ctx->err = "field outside point_step"; return SLO_E_ARG; }
    if (L.off_ring >= 0 && (uint64_t)L.off_ring + 2 > L.point_step) { ctx->err = "ring outside point_step"; return SLO_E_ARG; }
    SLO_CHECK(hipSetDevice(ctx->dev));
    const int P = ctx->cfg.max_points;
    const bool aligned = ((uintptr_t)d_bytes % 4 == 0) && msg_stride % 4 == 0 && L.point_step % 4 == 0 &&
                         (L.off_x < 0 || L.off_x % 4 == 0) && (L.off_y < 0 || L.off_y % 4 == 0) &&
                         (L.off_z < 0 || L.off_z % 4 == 0) && (L.off_intensity < 0 || L.off_intensity % 4 == 0);
    const dim3 grid((P + 255) / 256, ctx->S);
    k_pc2_unpack<<<grid, 256, 0, ctx->stream>>>(d_bytes, msg_stride, d_dims, L, P, aligned, (float4*)d_points,
                                                d_counts, d_rings, ctx->v.st);
    SLO_CHECK(hipGetLastError());
    return SLO_OK;
}

}  // extern "C"
