// orbx_frame_aux.hip -- the per-frame neighbours of the front end (SURVEY.md
// §8 f4) on gfx950, with their C ABI (include/orbx.h):
//   - MapPoint::ComputeDistinctiveDescriptors (MapPoint.cc:288-361): wave per
//     map point, medians by bisection over the distance range;
//   - Frame::UndistortKeyPoints (Frame.cc:438-469) = cv::undistortPoints with
//     R = I, P = K (OpenCV 3.2, double, 5 fixed iterations): thread per point;
//   - cvtColor *2GRAY for 8U (Tracking.cc:179-264): 14-bit fixed point,
//     4 pixels per thread;
//   - Mat::convertTo(CV_32F, 1/DepthMapFactor) of 16U depth (Tracking.cc:
//     228-229): 4 pixels per thread.
#include <hip/hip_runtime.h>

#include <climits>

#include "orbx_device.h"
#include "orbx_wave.h"
#include "orbx_ws.h"

namespace orbx {
namespace {

constexpr int kDT = 256;   // 4 waves, a map point each
constexpr int kDRows = 128;  // descriptors of a point staged in LDS (more: read from L2)

__device__ inline int hamming_rr(const uint4 a0, const uint4 a1, const uint4 b0, const uint4 b1) {
    return __popc(a0.x ^ b0.x) + __popc(a0.y ^ b0.y) + __popc(a0.z ^ b0.z) + __popc(a0.w ^ b0.w) +
           __popc(a1.x ^ b1.x) + __popc(a1.y ^ b1.y) + __popc(a1.z ^ b1.z) + __popc(a1.w ^ b1.w);
}

// The reference fills the N x N distance matrix, sorts each row and takes
// element (size_t)(0.5 * (N - 1)); the least median wins, first on ties.
// Here lane i finds its row's k-th smallest distance by bisection over
// [0, 256]: the smallest v with #{j : d(i, j) <= v} >= k + 1.
__global__ __launch_bounds__(kDT) void k_distinctive(const uint8_t *desc, const int32_t *offsets, int np,
                                                     int32_t *best) {
    __shared__ uint4 rows[kDT / 64][kDRows][2];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int p = blockIdx.x * (kDT / 64) + wave;
    if (p >= np) return;   // whole wave leaves together
    const int o = offsets[p], N = offsets[p + 1] - o;
    if (N <= 0) {
        if (lane == 0) best[p] = -1;
        return;
    }
    const uint4 *g = reinterpret_cast<const uint4 *>(desc + 32 * (int64_t)o);
    const bool staged = N <= kDRows;
    if (staged)
        for (int r = lane; r < N; r += 64) { rows[wave][r][0] = g[2 * r]; rows[wave][r][1] = g[2 * r + 1]; }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront", "local");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront", "local");
    const int k = (int)(0.5 * (double)(N - 1));   // the index the reference reads, truncated
    uint32_t keymin = ~0u;
    for (int i0 = 0; i0 < N; i0 += 64) {
        const int i = i0 + lane;
        uint32_t key = ~0u;
        if (i < N) {
            const uint4 a0 = staged ? rows[wave][i][0] : g[2 * i], a1 = staged ? rows[wave][i][1] : g[2 * i + 1];
            int lo = 0, hi = 256;
            while (lo < hi) {
                const int mid = (lo + hi) >> 1;
                int cnt = 0;
                for (int j = 0; j < N; ++j) {
                    const uint4 b0 = staged ? rows[wave][j][0] : g[2 * j], b1 = staged ? rows[wave][j][1] : g[2 * j + 1];
                    cnt += hamming_rr(a0, a1, b0, b1) <= mid;
                }
                if (cnt >= k + 1) hi = mid; else lo = mid + 1;
            }
            key = ((uint32_t)lo << 16) | (uint32_t)i;
        }
        keymin = min(keymin, wave_min_u32(key));
    }
    if (lane == 0) best[p] = (int32_t)(keymin & 0xFFFF);
}

struct UndistParams {
    double k[8];
    double fx, fy, cx, cy, ifx, ify;
    double RR[9];
};

__global__ void k_undistort(const float *xy, int n, UndistParams u, float *out) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const double *k = u.k;
    double x = xy[2 * i], y = xy[2 * i + 1], x0, y0;
    x0 = x = __dmul_rn(__dsub_rn(x, u.cx), u.ifx);
    y0 = y = __dmul_rn(__dsub_rn(y, u.cy), u.ify);
    for (int j = 0; j < 5; j++) {
        const double r2 = __dadd_rn(__dmul_rn(x, x), __dmul_rn(y, y));
        const double num = __dadd_rn(1.0, __dmul_rn(__dadd_rn(__dmul_rn(__dadd_rn(__dmul_rn(k[7], r2), k[6]), r2), k[5]), r2));
        const double den = __dadd_rn(1.0, __dmul_rn(__dadd_rn(__dmul_rn(__dadd_rn(__dmul_rn(k[4], r2), k[1]), r2), k[0]), r2));
        const double icdist = __ddiv_rn(num, den);
        const double deltaX = __dadd_rn(__dmul_rn(__dmul_rn(__dmul_rn(2.0, k[2]), x), y),
                                        __dmul_rn(k[3], __dadd_rn(r2, __dmul_rn(__dmul_rn(2.0, x), x))));
        const double deltaY = __dadd_rn(__dmul_rn(k[2], __dadd_rn(r2, __dmul_rn(__dmul_rn(2.0, y), y))),
                                        __dmul_rn(__dmul_rn(__dmul_rn(2.0, k[3]), x), y));
        x = __dmul_rn(__dsub_rn(x0, deltaX), icdist);
        y = __dmul_rn(__dsub_rn(y0, deltaY), icdist);
    }
    const double *R = u.RR;
    const double xx = __dadd_rn(__dadd_rn(__dmul_rn(R[0], x), __dmul_rn(R[1], y)), R[2]);
    const double yy = __dadd_rn(__dadd_rn(__dmul_rn(R[3], x), __dmul_rn(R[4], y)), R[5]);
    const double ww = __ddiv_rn(1.0, __dadd_rn(__dadd_rn(__dmul_rn(R[6], x), __dmul_rn(R[7], y)), R[8]));
    out[2 * i] = (float)__dmul_rn(xx, ww);
    out[2 * i + 1] = (float)__dmul_rn(yy, ww);
}

// 4 gray pixels per thread; grid.y = frame.
__global__ void k_cvt_gray(const uint8_t *src, int64_t sfs, int spitch, int cn, int rgb, int w, int h,
                           uint8_t *dst, int64_t dfs, int dpitch) {
    const int x4 = (blockIdx.x * blockDim.x + threadIdx.x) * 4;
    const int y = blockIdx.z;
    if (x4 >= w || y >= h) return;
    const uint8_t *s = src + blockIdx.y * sfs + (int64_t)y * spitch + (int64_t)x4 * cn;
    uint8_t *d = dst + blockIdx.y * dfs + (int64_t)y * dpitch + x4;
    const int c0 = rgb ? 4899 : 1868, c2 = rgb ? 1868 : 4899;   // src[0] / src[2] weights (R2Y / B2Y)
    const int m = min(4, w - x4);
    for (int t = 0; t < m; ++t) {
        const uint8_t *q = s + t * cn;
        d[t] = (uint8_t)((q[0] * c0 + q[1] * 9617 + q[2] * c2 + (1 << 13)) >> 14);
    }
}

__global__ void k_depth_float(const uint16_t *src, int64_t sfs, int spitch, int w, int h, float scale, float *dst,
                              int64_t dfs, int dpitch) {
    const int x4 = (blockIdx.x * blockDim.x + threadIdx.x) * 4;
    const int y = blockIdx.z;
    if (x4 >= w || y >= h) return;
    const uint16_t *s = reinterpret_cast<const uint16_t *>(reinterpret_cast<const uint8_t *>(src) + blockIdx.y * sfs +
                                                           (int64_t)y * spitch) + x4;
    float *d = reinterpret_cast<float *>(reinterpret_cast<uint8_t *>(dst) + blockIdx.y * dfs + (int64_t)y * dpitch) + x4;
    const int m = min(4, w - x4);
    for (int t = 0; t < m; ++t) d[t] = __fmul_rn((float)s[t], scale);
}

bool make_undist(const float *K, const float *dist, int ncoef, UndistParams &u) {
    if (!K || !dist || ncoef < 4 || ncoef > 8) return false;
    for (int i = 0; i < 8; ++i) u.k[i] = i < ncoef ? (double)dist[i] : 0.0;
    u.fx = K[0]; u.fy = K[4]; u.cx = K[2]; u.cy = K[5];
    u.ifx = 1. / u.fx;
    u.ify = 1. / u.fy;
    for (int i = 0; i < 9; ++i) u.RR[i] = K[i];   // P * I
    return true;
}

hipError_t launch_pixels(bool depth, const void *src, int64_t sfs, int spitch, int cn, int rgb, int w, int h,
                         int batch, float scale, void *dst, int64_t dfs, int dpitch, hipStream_t st) {
    const int threads = (w + 3) / 4;
    const dim3 grid((threads + 255) / 256, batch, h);
    if (depth)
        hipLaunchKernelGGL(k_depth_float, grid, dim3(256), 0, st, static_cast<const uint16_t *>(src), sfs, spitch, w,
                           h, scale, static_cast<float *>(dst), dfs, dpitch);
    else
        hipLaunchKernelGGL(k_cvt_gray, grid, dim3(256), 0, st, static_cast<const uint8_t *>(src), sfs, spitch, cn,
                           rgb, w, h, static_cast<uint8_t *>(dst), dfs, dpitch);
    return hipGetLastError();
}

}  // namespace
}  // namespace orbx

using namespace orbx;

extern "C" {

int orbx_distinctive_descriptors_device(const uint8_t *d_desc, const int32_t *d_offsets, int npoints, int32_t *d_best,
                                        void *stream) {
    if (npoints < 0 || (npoints && (!d_desc || !d_offsets || !d_best))) return ORBX_EINVAL;
    if (npoints == 0) return ORBX_OK;
    hipLaunchKernelGGL(k_distinctive, dim3((npoints + kDT / 64 - 1) / (kDT / 64)), dim3(kDT), 0,
                       static_cast<hipStream_t>(stream), d_desc, d_offsets, npoints, d_best);
    return hipGetLastError() == hipSuccess ? ORBX_OK : ORBX_EIO;
}

int orbx_distinctive_descriptors(int device, const uint8_t *desc, const int32_t *offsets, int npoints, int32_t *best) {
    if (npoints < 0 || !offsets || (npoints && !best)) return ORBX_EINVAL;
    if (offsets[0] != 0) return ORBX_EINVAL;
    for (int p = 0; p < npoints; ++p)
        if (offsets[p + 1] < offsets[p] || offsets[p + 1] - offsets[p] > 65535) return ORBX_EINVAL;
    const int total = offsets[npoints];
    if (total && !desc) return ORBX_EINVAL;
    if (npoints == 0) return ORBX_OK;
    if (hipSetDevice(device) != hipSuccess) return ORBX_ENODEV;
    Layout L;
    const size_t o_d = L.add(32 * (size_t)std::max(total, 1)), o_o = L.add(4 * (size_t)(npoints + 1));
    const size_t in_bytes = L.size;
    const size_t o_b = L.add(4 * (size_t)npoints);
    CallWs &ws = call_ws(device);
    std::lock_guard<std::mutex> lock(ws.mu);
    int rc = ws_reserve(ws, L.size);
    if (rc) return rc;
    put(ws, o_d, desc, 32 * (size_t)total);
    put(ws, o_o, offsets, 4 * (size_t)(npoints + 1));
    uint8_t *D = ws.dev;
    if (hipMemcpyAsync(D, ws.host, in_bytes, hipMemcpyHostToDevice, ws.st) != hipSuccess) return ORBX_EIO;
    rc = orbx_distinctive_descriptors_device(D + o_d, at<int32_t>(D, o_o), npoints, at<int32_t>(D, o_b), ws.st);
    if (rc) return rc;
    if (hipMemcpyAsync(ws.host + o_b, D + o_b, 4 * (size_t)npoints, hipMemcpyDeviceToHost, ws.st) != hipSuccess ||
        hipStreamSynchronize(ws.st) != hipSuccess)
        return ORBX_EIO;
    get(ws, o_b, best, 4 * (size_t)npoints);
    return ORBX_OK;
}

int orbx_undistort_points_device(const float *d_xy, int n, const float *K, const float *dist, int ncoef,
                                 float *d_xy_un, void *stream) {
    UndistParams u;
    if (n < 0 || (n && (!d_xy || !d_xy_un)) || !make_undist(K, dist, ncoef, u)) return ORBX_EINVAL;
    if (n == 0) return ORBX_OK;
    hipStream_t st = static_cast<hipStream_t>(stream);
    if (dist[0] == 0.0f)   // Frame.cc:441: mvKeysUn = mvKeys
        return d_xy == d_xy_un || hipMemcpyAsync(d_xy_un, d_xy, 8 * (size_t)n, hipMemcpyDeviceToDevice, st) ==
                                      hipSuccess ? ORBX_OK : ORBX_EIO;
    hipLaunchKernelGGL(k_undistort, dim3((n + 255) / 256), dim3(256), 0, st, d_xy, n, u, d_xy_un);
    return hipGetLastError() == hipSuccess ? ORBX_OK : ORBX_EIO;
}

int orbx_undistort_keypoints(int device, const orbx_keypoint *kps, int n, const float *K, const float *dist,
                             int ncoef, orbx_keypoint *kps_un) {
    UndistParams u;
    if (n < 0 || (n && (!kps || !kps_un)) || !make_undist(K, dist, ncoef, u)) return ORBX_EINVAL;
    if (kps_un != kps) std::memcpy(kps_un, kps, sizeof(orbx_keypoint) * (size_t)n);   // kp = mvKeys[i]
    if (n == 0 || dist[0] == 0.0f) return ORBX_OK;
    if (hipSetDevice(device) != hipSuccess) return ORBX_ENODEV;
    Layout L;
    const size_t o_in = L.add(8 * (size_t)n), o_out = L.add(8 * (size_t)n);
    CallWs &ws = call_ws(device);
    std::lock_guard<std::mutex> lock(ws.mu);
    int rc = ws_reserve(ws, L.size);
    if (rc) return rc;
    float *h_in = at<float>(ws.host, o_in);
    for (int i = 0; i < n; ++i) { h_in[2 * i] = kps[i].x; h_in[2 * i + 1] = kps[i].y; }
    uint8_t *D = ws.dev;
    if (hipMemcpyAsync(D + o_in, h_in, 8 * (size_t)n, hipMemcpyHostToDevice, ws.st) != hipSuccess) return ORBX_EIO;
    hipLaunchKernelGGL(k_undistort, dim3((n + 255) / 256), dim3(256), 0, ws.st, at<float>(D, o_in), n, u,
                       at<float>(D, o_out));
    if (hipGetLastError() != hipSuccess ||
        hipMemcpyAsync(ws.host + o_out, D + o_out, 8 * (size_t)n, hipMemcpyDeviceToHost, ws.st) != hipSuccess ||
        hipStreamSynchronize(ws.st) != hipSuccess)
        return ORBX_EIO;
    const float *h_out = at<float>(ws.host, o_out);
    for (int i = 0; i < n; ++i) { kps_un[i].x = h_out[2 * i]; kps_un[i].y = h_out[2 * i + 1]; }
    return ORBX_OK;
}

int orbx_cvt_gray_device(const uint8_t *d_src, int64_t src_frame_stride, int src_pitch, int channels, int rgb, int w,
                         int h, int batch, uint8_t *d_dst, int64_t dst_frame_stride, int dst_pitch, void *stream) {
    if ((channels != 3 && channels != 4) || w <= 0 || h <= 0 || batch <= 0 || batch > 65535 || !d_src || !d_dst ||
        src_pitch < channels * w || dst_pitch < w)
        return ORBX_EINVAL;
    return launch_pixels(false, d_src, src_frame_stride, src_pitch, channels, rgb ? 1 : 0, w, h, batch, 0.f, d_dst,
                         dst_frame_stride, dst_pitch, static_cast<hipStream_t>(stream)) == hipSuccess ? ORBX_OK
                                                                                                      : ORBX_EIO;
}

int orbx_cvt_gray(int device, const uint8_t *src, int w, int h, size_t pitch, int channels, int rgb, uint8_t *dst,
                  size_t dst_pitch) {
    if ((channels != 3 && channels != 4) || w <= 0 || h <= 0 || !src || !dst || pitch < (size_t)channels * w ||
        dst_pitch < (size_t)w)
        return ORBX_EINVAL;
    if (hipSetDevice(device) != hipSuccess) return ORBX_ENODEV;
    const size_t sp = (size_t)channels * w;
    Layout L;
    const size_t o_s = L.add(sp * h), o_d = L.add((size_t)w * h);
    CallWs &ws = call_ws(device);
    std::lock_guard<std::mutex> lock(ws.mu);
    int rc = ws_reserve(ws, L.size);
    if (rc) return rc;
    for (int y = 0; y < h; ++y) std::memcpy(ws.host + o_s + sp * y, src + pitch * y, sp);
    uint8_t *D = ws.dev;
    if (hipMemcpyAsync(D + o_s, ws.host + o_s, sp * h, hipMemcpyHostToDevice, ws.st) != hipSuccess ||
        launch_pixels(false, D + o_s, 0, (int)sp, channels, rgb ? 1 : 0, w, h, 1, 0.f, D + o_d, 0, w, ws.st) !=
            hipSuccess ||
        hipMemcpyAsync(ws.host + o_d, D + o_d, (size_t)w * h, hipMemcpyDeviceToHost, ws.st) != hipSuccess ||
        hipStreamSynchronize(ws.st) != hipSuccess)
        return ORBX_EIO;
    for (int y = 0; y < h; ++y) std::memcpy(dst + dst_pitch * y, ws.host + o_d + (size_t)w * y, (size_t)w);
    return ORBX_OK;
}

int orbx_depth_to_float_device(const uint16_t *d_src, int64_t src_frame_stride, int src_pitch, int w, int h,
                               int batch, float scale, float *d_dst, int64_t dst_frame_stride, int dst_pitch,
                               void *stream) {
    if (w <= 0 || h <= 0 || batch <= 0 || batch > 65535 || !d_src || !d_dst || src_pitch < 2 * w ||
        dst_pitch < 4 * w || (src_pitch & 1) || (dst_pitch & 3))
        return ORBX_EINVAL;
    return launch_pixels(true, d_src, src_frame_stride, src_pitch, 1, 0, w, h, batch, scale, d_dst, dst_frame_stride,
                         dst_pitch, static_cast<hipStream_t>(stream)) == hipSuccess ? ORBX_OK : ORBX_EIO;
}

}  // extern "C"
