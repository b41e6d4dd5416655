// orbx_ba.hip -- Optimizer::LocalBundleAdjustment (Optimizer.cc:517-900) on
// gfx950: g2o's Levenberg-Marquardt (optimization_algorithm_levenberg.cpp:
// 60-160) over a BlockSolver_6_3 (block_solver.hpp: buildSystem, Schur
// complement :354-484) with EdgeSE3ProjectXYZ / EdgeStereoSE3ProjectXYZ
// (types_six_dof_expmap.cpp:109-230) and Huber kernels (robust_kernel_impl.
// cpp:78-91).  SURVEY.md §8 f2, config C4.
//
// Device work per LM trial, all FP64:
//   k_ba_errors        thread per edge: error, chi2, Huber rho (computeActiveErrors)
//   k_ba_linearize     thread per edge: Jacobians and the edge's J^T W J / J^T W r blocks
//   k_ba_gather_rows / k_ba_stream_sums
//                      Hpp / bp of each free camera (and the reduced right-hand side
//                      bp - sum B Dinv bl) as sums over its edges in edge order: the
//                      records gathered into list order, then a workgroup per camera adds
//   k_ba_reduce        wave per point: Hll / bl, edge order
//   k_ba_point         thread per point: (Hll + lambda I)^-1 and Dinv bl
//   k_ba_point_edges   thread per edge: B Dinv and B Dinv bl
//   k_ba_pair_terms    thread per (shared point, entry) of every camera pair: B_i Dinv B_j^T terms
//   k_ba_pairs_sum     workgroup per camera pair: S_ij -= its terms in point order (pairs listed once
//                      per set of active edges); k_ba_pairs merge walk for repeated observations
//   k_ba_chol_lds      one workgroup: blocked dense Cholesky of the reduced camera system and
//                      the solves (k_ba_chol beyond 128 unknowns)
//   k_ba_chol_fast     fast mode: the augmented system on the FP64 matrix cores, tiles resident in
//                      the accumulators, a division-free panel chain (<= 126 unknowns)
//   k_ba_backsub_terms / k_ba_backsub
//                      xl = Dinv (bl - sum_e B_e^T xp): per-edge terms, then thread per point
//   k_ba_update        poses exp(dx) * T (SE3Quat), points += dx
// Every sum runs in a fixed order (edge order per vertex, ascending point per
// camera pair, ascending column in the Cholesky), so a run is deterministic
// and matches the oracle's CPU restatement of the same order.  g2o's own order
// is unspecified (it sorts edges with equal ids), so parity with it is to
// rounding only.  The LM control (lambda, rho, trials, termination) runs on
// the host as in the reference, with one stream synchronisation per trial
// (lm_optimize).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cfloat>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cmath>
#include <cstring>
#include <mutex>
#include <set>
#include <type_traits>
#include <vector>

#include "orbx_device.h"
#include "orbx_wave.h"
#include "orbx_ws.h"

namespace orbx {
namespace {

struct Pose {      // SE3Quat: q = (x, y, z, w), t
    double q[4];
    double t[3];
    int32_t free_idx;   // -1: fixed
    int32_t pad;
};

struct EdgeD {     // one observation, device copy
    int32_t cam, point, stereo, pad;
    double obs[3];
    double omega;   // information = omega * I
    double fx, fy, cx, cy, bf;
    double delta;   // Huber delta
};

struct EdgeOut {   // per edge, per linearization
    double hpp[36], hll[9], hpl[18];   // hpl: 6 x 3 (pose rows, point cols)
    double bp[6], bl[3];
};

// Eigen's q * v (Quaternion::_transformVector): uv = 2 (q.vec x v); v + w uv + q.vec x uv
__host__ __device__ inline void quat_rotate(const double *q, const double *v, double *o) {
    double uv[3] = {q[1] * v[2] - q[2] * v[1], q[2] * v[0] - q[0] * v[2], q[0] * v[1] - q[1] * v[0]};
    for (int i = 0; i < 3; ++i) uv[i] = uv[i] + uv[i];
    const double c[3] = {q[1] * uv[2] - q[2] * uv[1], q[2] * uv[0] - q[0] * uv[2], q[0] * uv[1] - q[1] * uv[0]};
    for (int i = 0; i < 3; ++i) o[i] = v[i] + q[3] * uv[i] + c[i];
}

__host__ __device__ inline void se3_map(const Pose &T, const double *X, double *o) {
    quat_rotate(T.q, X, o);
    for (int i = 0; i < 3; ++i) o[i] = o[i] + T.t[i];
}

// Eigen's Quaternion::toRotationMatrix
__host__ __device__ inline void quat_to_R(const double *q, double *R) {
    const double tx = 2 * q[0], ty = 2 * q[1], tz = 2 * q[2];
    const double twx = tx * q[3], twy = ty * q[3], twz = tz * q[3];
    const double txx = tx * q[0], txy = ty * q[0], txz = tz * q[0];
    const double tyy = ty * q[1], tyz = tz * q[1], tzz = tz * q[2];
    R[0] = 1 - (tyy + tzz); R[1] = txy - twz; R[2] = txz + twy;
    R[3] = txy + twz; R[4] = 1 - (txx + tzz); R[5] = tyz - twx;
    R[6] = txz - twy; R[7] = tyz + twx; R[8] = 1 - (txx + tyy);
}

// Eigen's Quaternion(const Matrix3&) (quaternion_base_assign_impl)
__host__ __device__ inline void R_to_quat(const double *m, double *q) {
    const double tr = m[0] + m[4] + m[8];
    if (tr > 0) {
        double t = sqrt(tr + 1.0);
        q[3] = 0.5 * t;
        t = 0.5 / t;
        q[0] = (m[7] - m[5]) * t;
        q[1] = (m[2] - m[6]) * t;
        q[2] = (m[3] - m[1]) * t;
    } else {
        int i = 0;
        if (m[4] > m[0]) i = 1;
        if (m[8] > m[3 * i + i]) i = 2;
        const int j = (i + 1) % 3, k = (j + 1) % 3;
        double t = sqrt(m[3 * i + i] - m[3 * j + j] - m[3 * k + k] + 1.0);
        q[i] = 0.5 * t;
        t = 0.5 / t;
        q[3] = (m[3 * k + j] - m[3 * j + k]) * t;
        q[j] = (m[3 * j + i] + m[3 * i + j]) * t;
        q[k] = (m[3 * k + i] + m[3 * i + k]) * t;
    }
}

// SE3Quat::normalizeRotation: w >= 0, unit norm
__host__ __device__ inline void quat_normalize(double *q) {
    if (q[3] < 0)
        for (int i = 0; i < 4; ++i) q[i] *= -1;
    const double n = sqrt(q[0] * q[0] + q[1] * q[1] + q[2] * q[2] + q[3] * q[3]);
    for (int i = 0; i < 4; ++i) q[i] = q[i] / n;
}

// Eigen's quaternion product a * b
__host__ __device__ inline void quat_mul(const double *a, const double *b, double *o) {
    o[3] = a[3] * b[3] - a[0] * b[0] - a[1] * b[1] - a[2] * b[2];
    o[0] = a[3] * b[0] + a[0] * b[3] + a[1] * b[2] - a[2] * b[1];
    o[1] = a[3] * b[1] + a[1] * b[3] + a[2] * b[0] - a[0] * b[2];
    o[2] = a[3] * b[2] + a[2] * b[3] + a[0] * b[1] - a[1] * b[0];
}

// error of an edge (computeError) and whether the point is in front
__device__ inline void edge_error(const EdgeD &e, const Pose &T, const double *X, double *err, bool *front) {
    double p[3];
    se3_map(T, X, p);
    *front = p[2] > 0.0;
    if (!e.stereo) {
        const double u = p[0] / p[2], v = p[1] / p[2];
        err[0] = e.obs[0] - (u * e.fx + e.cx);
        err[1] = e.obs[1] - (v * e.fy + e.cy);
        err[2] = 0;
    } else {
        const double invz = (double)(float)(1.0 / p[2]);   // const float invz = 1.0f/trans_xyz[2]
        const double r0 = p[0] * invz * e.fx + e.cx;
        const double r1 = p[1] * invz * e.fy + e.cy;
        err[0] = e.obs[0] - r0;
        err[1] = e.obs[1] - r1;
        err[2] = e.obs[2] - (r0 - e.bf * invz);
    }
}

// One edge's error at the current estimate: front flag, and for an active
// edge (computeActiveErrors) err, chi2, rho; returns rho0 (0 if inactive or
// front_only)
__device__ inline double ba_edge_error(int i, const Pose *poses, const double *pts, const EdgeD *edges,
                                       const uint8_t *active, int robust, int front_only, double *err_out,
                                       double *chi2_out, double *rho_out, uint8_t *front_out, double *rho0_out) {
    const EdgeD e = edges[i];
    double err[3];
    bool front;
    edge_error(e, poses[e.cam], pts + 3 * (int64_t)e.point, err, &front);
    front_out[i] = front;   // isDepthPositive() at the current estimate
    if (front_only || !active[i]) return 0.0;   // computeActiveErrors leaves inactive edges' errors as they were
    const int D = e.stereo ? 3 : 2;
    double chi2 = 0;
    for (int k = 0; k < D; ++k) chi2 = chi2 + err[k] * (e.omega * err[k]);
    double rho0 = chi2, rho1 = 1.0;
    if (robust) {
        const double dsqr = e.delta * e.delta;
        if (!(chi2 <= dsqr)) {
            const double s = sqrt(chi2);
            rho0 = 2 * s * e.delta - dsqr;
            rho1 = e.delta / s;
        }
    }
    for (int k = 0; k < 3; ++k) err_out[3 * (int64_t)i + k] = err[k];
    chi2_out[i] = chi2;
    rho_out[2 * (int64_t)i] = rho0;
    rho_out[2 * (int64_t)i + 1] = rho1;
    if (rho0_out) rho0_out[i] = rho0;   // (contiguous, for the host's ordered sum)
    return rho0;
}

// gate (optional): run only when *gate != 0 (a trial whose solve failed
// leaves the estimate and the errors alone)
__global__ void k_ba_errors(const Pose *poses, const double *pts, const EdgeD *edges, int ne, const uint8_t *active,
                            int robust, int front_only, double *err_out, double *chi2_out, double *rho_out,
                            uint8_t *front_out, double *rho0_out, const int *gate) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= ne || (gate && !*gate)) return;
    (void)ba_edge_error(i, poses, pts, edges, active, robust, front_only, err_out, chi2_out, rho_out, front_out,
                        rho0_out);
}

// One edge's blocks (D = 2 mono, 3 stereo: compile-time, so the Jacobians
// stay in registers), stored field by field into out
template <int D>
__device__ inline void linearize_edge(const EdgeD &e, const Pose &T, const double *p, double rho1, const double *err,
                                      double *out) {
    const double x = p[0], y = p[1], z = p[2], z_2 = z * z;
    double R[9];
    quat_to_R(T.q, R);
    double A[D][3], B[D][6];   // d e / d point, d e / d pose (rows: error components)
    if (D == 2) {
        const double tmp[2][3] = {{e.fx, 0, -x / z * e.fx}, {0, e.fy, -y / z * e.fy}};
        const double s = -1. / z;
#pragma unroll
        for (int r = 0; r < 2; ++r)
#pragma unroll
            for (int c = 0; c < 3; ++c) {
                double acc = 0;
#pragma unroll
                for (int k = 0; k < 3; ++k) acc = acc + (s * tmp[r][k]) * R[3 * k + c];
                A[r][c] = acc;
            }
    } else {
#pragma unroll
        for (int c = 0; c < 3; ++c) {
            A[0][c] = -e.fx * R[c] / z + e.fx * x * R[6 + c] / z_2;
            A[1][c] = -e.fy * R[3 + c] / z + e.fy * y * R[6 + c] / z_2;
            A[D - 1][c] = A[0][c] - e.bf * R[6 + c] / z_2;
        }
    }
    B[0][0] = x * y / z_2 * e.fx;
    B[0][1] = -(1 + (x * x / z_2)) * e.fx;
    B[0][2] = y / z * e.fx;
    B[0][3] = -1. / z * e.fx;
    B[0][4] = 0;
    B[0][5] = x / z_2 * e.fx;
    B[1][0] = (1 + y * y / z_2) * e.fy;
    B[1][1] = -x * y / z_2 * e.fy;
    B[1][2] = -x / z * e.fy;
    B[1][3] = 0;
    B[1][4] = -1. / z * e.fy;
    B[1][5] = y / z_2 * e.fy;
    if (D == 3) {
        B[D - 1][0] = B[0][0] - e.bf * y / z_2;
        B[D - 1][1] = B[0][1] + e.bf * x / z_2;
        B[D - 1][2] = B[0][2];
        B[D - 1][3] = B[0][3];
        B[D - 1][4] = 0;
        B[D - 1][5] = B[0][5] - e.bf / z_2;
    }
    const double w = rho1 * e.omega;   // robustInformation = rho[1] * information (rho1 = 1 without a kernel)
    double omr[D];
#pragma unroll
    for (int k = 0; k < D; ++k) omr[k] = -(e.omega * err[k]) * rho1;
    double *hpp = out, *hll = out + 36, *hpl = out + 45, *bp = out + 63, *bl = out + 69;   // EdgeOut's fields
#pragma unroll
    for (int a = 0; a < 3; ++a)
#pragma unroll
        for (int b = 0; b < 3; ++b) {
            double acc = 0;
#pragma unroll
            for (int k = 0; k < D; ++k) acc = acc + (A[k][a] * w) * A[k][b];
            hll[3 * a + b] = acc;
        }
    const bool pose_free = T.free_idx >= 0;
#pragma unroll
    for (int a = 0; a < 6; ++a) {
#pragma unroll
        for (int b = 0; b < 6; ++b) {
            double acc = 0;
            if (pose_free)
#pragma unroll
                for (int k = 0; k < D; ++k) acc = acc + (B[k][a] * w) * B[k][b];
            hpp[6 * a + b] = acc;
        }
#pragma unroll
        for (int c = 0; c < 3; ++c) {   // (A^T W B)^T: pose row a, point column c
            double acc = 0;
            if (pose_free)
#pragma unroll
                for (int k = 0; k < D; ++k) acc = acc + (A[k][c] * w) * B[k][a];
            hpl[3 * a + c] = acc;
        }
        double acc = 0;
        if (pose_free)
#pragma unroll
            for (int k = 0; k < D; ++k) acc = acc + B[k][a] * omr[k];
        bp[a] = acc;
    }
#pragma unroll
    for (int c = 0; c < 3; ++c) {
        double acc = 0;
#pragma unroll
        for (int k = 0; k < D; ++k) acc = acc + A[k][c] * omr[k];
        bl[c] = acc;
    }
}

// gate (fast mode's speculative build, lm_optimize): run only if *gate != 0
__global__ void k_ba_linearize(const Pose *poses, const double *pts, const EdgeD *edges, int ne, const uint8_t *active,
                               const double *err_in, const double *rho_in, EdgeOut *out, const int *gate) {
    static_assert(sizeof(EdgeOut) == 72 * sizeof(double), "EdgeOut layout");
    if (gate && !*gate) return;
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= ne || !active[i]) return;
    const EdgeD e = edges[i];
    const Pose T = poses[e.cam];
    double p[3];
    se3_map(T, pts + 3 * (int64_t)e.point, p);
    const double rho1 = rho_in[2 * (int64_t)i + 1];
    const double *err = err_in + 3 * (int64_t)i;
    double *o = reinterpret_cast<double *>(out + i);
    if (e.stereo) linearize_edge<3>(e, T, p, rho1, err, o);
    else linearize_edge<2>(e, T, p, rho1, err, o);
}

// Vertex blocks: wave per vertex, lane = one matrix entry, edges in order.
// kind 0: cameras (36 + 6 entries from hpp / bp), 1: points (9 + 3 from hll / bl).
__global__ void k_ba_reduce(const EdgeOut *eo, const int32_t *offs, const int32_t *list, const uint8_t *active,
                            int nv, int kind, double *H, double *b, const int *gate) {
    if (gate && !*gate) return;
    const int lane = threadIdx.x & 63;
    const int v = blockIdx.x * (blockDim.x / 64) + (threadIdx.x >> 6);
    if (v >= nv) return;
    const int nh = kind ? 9 : 36, nb = kind ? 3 : 6;
    if (lane >= nh + nb) return;
    // the field this lane sums, as a double offset into EdgeOut
    const int fo = lane < nh ? (kind ? 36 + lane : lane) : (kind ? 63 + 6 + lane - nh : 63 + lane - nh);
    const double *base = reinterpret_cast<const double *>(eo) + fo;
    constexpr int kEo = sizeof(EdgeOut) / sizeof(double);
    double acc = 0;
    // 8 edges' loads in flight, then their sum in edge order
    int t = offs[v];
    const int te = offs[v + 1];
    for (; t + 8 <= te; t += 8) {
        int ei[8];
        double val[8];
        uint8_t a[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) ei[j] = list[t + j];
#pragma unroll
        for (int j = 0; j < 8; ++j) { a[j] = active[ei[j]]; val[j] = base[(int64_t)ei[j] * kEo]; }
#pragma unroll
        for (int j = 0; j < 8; ++j)
            if (a[j]) acc = acc + val[j];
    }
    if (t < te) {   // the tail too: its loads in flight together, then added in edge order
        const int nr = te - t;
        int ei[8];
        double val[8];
        bool a[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) ei[j] = list[t + (j < nr ? j : 0)];
#pragma unroll
        for (int j = 0; j < 8; ++j) { a[j] = j < nr && active[ei[j]]; val[j] = base[(int64_t)ei[j] * kEo]; }
#pragma unroll
        for (int j = 0; j < 8; ++j)
            if (a[j]) acc = acc + val[j];
    }
    if (lane < nh) H[(int64_t)v * nh + lane] = acc;
    else b[(int64_t)v * nb + lane - nh] = acc;
}

// Per point: Dinv = (Hll + lambda I)^-1 (Eigen's 3x3 cofactor inverse),
// db = Dinv bl, then for each of its active free-camera edges B Dinv and B db.
__device__ inline double cof(const double *m, int i, int j) {
    const int i1 = (i + 1) % 3, i2 = (i + 2) % 3, j1 = (j + 1) % 3, j2 = (j + 2) % 3;
    return m[3 * i1 + j1] * m[3 * i2 + j2] - m[3 * i1 + j2] * m[3 * i2 + j1];
}

__global__ void k_ba_point(const double *Hll, const double *bl, int npt, double lambda, double *dinv_out,
                           double *db_out, double *lu_out) {
    const int pt = blockIdx.x * blockDim.x + threadIdx.x;
    if (pt >= npt) return;
    double m[9];
    for (int k = 0; k < 9; ++k) m[k] = Hll[9 * (int64_t)pt + k];
    for (int k = 0; k < 3; ++k) m[4 * k] = m[4 * k] + lambda;
    const double c0 = cof(m, 0, 0), c1 = cof(m, 1, 0), c2 = cof(m, 2, 0);
    const double det = c0 * m[0] + c1 * m[3] + c2 * m[6];
    const double invdet = 1.0 / det;
    double D[9];
    D[0] = c0 * invdet; D[1] = c1 * invdet; D[2] = c2 * invdet;
    D[3] = cof(m, 0, 1) * invdet; D[4] = cof(m, 1, 1) * invdet; D[5] = cof(m, 2, 1) * invdet;
    D[6] = cof(m, 0, 2) * invdet; D[7] = cof(m, 1, 2) * invdet; D[8] = cof(m, 2, 2) * invdet;
    for (int k = 0; k < 9; ++k) dinv_out[9 * (int64_t)pt + k] = D[k];
    for (int r = 0; r < 3; ++r) {
        double acc = 0;
        for (int c = 0; c < 3; ++c) acc = acc + D[3 * r + c] * bl[3 * (int64_t)pt + c];
        db_out[3 * (int64_t)pt + r] = acc;
    }
    if (lu_out) {   // (fast mode's dense Schur product) m = L L^T: L^-1 (lower, six) and u = L^-1 bl
        const double l00 = sqrt(m[0]), l10 = m[3] / l00, l20 = m[6] / l00;
        const double l11 = sqrt(m[4] - l10 * l10), l21 = (m[7] - l20 * l10) / l11;
        const double l22 = sqrt(m[8] - l20 * l20 - l21 * l21);
        const double i00 = 1.0 / l00, i11 = 1.0 / l11, i22 = 1.0 / l22;
        const double i10 = -l10 * i00 * i11, i21 = -l21 * i11 * i22, i20 = -(l20 * i00 + l21 * i10) * i22;
        const double *b = bl + 3 * (int64_t)pt;
        double *o = lu_out + 9 * (int64_t)pt;
        o[0] = i00; o[1] = i10; o[2] = i11; o[3] = i20; o[4] = i21; o[5] = i22;
        o[6] = i00 * b[0];
        o[7] = i10 * b[0] + i11 * b[1];
        o[8] = i20 * b[0] + i21 * b[1] + i22 * b[2];
    }
}

// per usable edge: B Dinv (6x3) and B Dinv bl (6) of its point (thread per
// edge, so the work spreads over every edge, not over the points' lists)
__global__ void k_ba_point_edges(const EdgeOut *eo, const int32_t *epoint, const uint8_t *usable, int ne,
                                 const double *dinv, const double *db, double *bdinv, double *bdb) {
    const int ei = blockIdx.x * blockDim.x + threadIdx.x;
    if (ei >= ne || !usable[ei]) return;
    const int pt = epoint[ei];
    double D[9], d3[3];
    for (int k = 0; k < 9; ++k) D[k] = dinv[9 * (int64_t)pt + k];
    for (int k = 0; k < 3; ++k) d3[k] = db[3 * (int64_t)pt + k];
    const double *B = eo[ei].hpl;
    for (int r = 0; r < 6; ++r) {
        for (int c = 0; c < 3; ++c) {
            double acc = 0;
            for (int k = 0; k < 3; ++k) acc = acc + B[3 * r + k] * D[3 * k + c];
            bdinv[18 * (int64_t)ei + 3 * r + c] = acc;
        }
        double acc = 0;
        for (int k = 0; k < 3; ++k) acc = acc + B[3 * r + k] * d3[k];
        bdb[6 * (int64_t)ei + r] = acc;
    }
}

__global__ void k_ba_pairs(const int2 *pairs, int npairs, const int32_t *coffs, const int32_t *clist,
                           const int32_t *epoint, const EdgeOut *eo, const double *bdinv, const double *Hpp,
                           double lambda, int nf, double *S) {
    const int lane = threadIdx.x & 63;
    const int pi = blockIdx.x * (blockDim.x / 64) + (threadIdx.x >> 6);
    if (pi >= npairs || lane >= 36) return;
    const int i1 = pairs[pi].x, i2 = pairs[pi].y;
    const int r = lane / 6, c = lane % 6;
    double acc = 0;
    if (i1 == i2) {
        acc = Hpp[36 * (int64_t)i1 + lane];
        if (r == c) acc = acc + lambda;
    }
    int a = coffs[i1], ae = coffs[i1 + 1], b = coffs[i2], be = coffs[i2 + 1];
    while (a < ae && b < be) {
        const int pa = epoint[clist[a]], pb = epoint[clist[b]];
        if (pa < pb) { ++a; continue; }
        if (pb < pa) { ++b; continue; }
        const int e1 = clist[a], e2 = clist[b];
        double s = 0;
        for (int k = 0; k < 3; ++k) s = s + bdinv[18 * (int64_t)e1 + 3 * r + k] * eo[e2].hpl[3 * c + k];
        acc = acc - s;
        ++a;
        ++b;
    }
    const int n = 6 * nf;
    S[(int64_t)(6 * i1 + r) * n + 6 * i2 + c] = acc;
    S[(int64_t)(6 * i2 + c) * n + 6 * i1 + r] = acc;   // mirror (the solver reads the full matrix)
}

// The shared points of each camera pair as (edge of i1, edge of i2) in
// ascending point order, found lane-parallel: a wave walks camera i1's list
// 64 entries at a time and looks each point up in camera i2's point ->
// list-position map (cmap, -1: not observed; needs each (camera, point)
// observed at most once, checked on the host).  A count pass
// (moffs == nullptr: counts out) and a fill pass at the scanned offsets.
// Built once per set of active edges; the per-trial Schur pass then streams
// the list with independent loads.
__global__ __launch_bounds__(256) void k_ba_pair_matches(const int2 *pairs, int npairs, const int32_t *coffs,
                                                         const int32_t *clist, const int32_t *epoint,
                                                         const int32_t *cmap, int npt, const int32_t *moffs,
                                                         int32_t *counts, int2 *mlist) {
    const int lane = threadIdx.x & 63, pi = blockIdx.x * 4 + (threadIdx.x >> 6);
    if (pi >= npairs) return;
    const int i1 = pairs[pi].x, i2 = pairs[pi].y;
    const int32_t *map2 = cmap + (int64_t)i2 * npt;
    int at = moffs ? moffs[pi] : 0;
    for (int a0 = coffs[i1]; a0 < coffs[i1 + 1]; a0 += 64) {
        const int a = a0 + lane;
        int e1 = -1, e2 = -1;
        if (a < coffs[i1 + 1]) {
            e1 = clist[a];
            const int pos = map2[epoint[e1]];
            if (pos >= 0) e2 = clist[pos];
        }
        const uint64_t m = __ballot(e2 >= 0);
        if (moffs && e2 >= 0)
            mlist[at + (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u))] =
                make_int2(e1, e2);
        at += __popcll(m);
    }
    if (!moffs && lane == 0) counts[pi] = at;
}

// point -> position in camera f's usable list (the map k_ba_pair_matches reads)
// (ids: the edge itself instead of its list position -- the fast mode's
// dense Schur product reads the map that way)
__global__ void k_ba_cmap(const int32_t *coffs, const int32_t *clist, const int32_t *epoint, int npt, int32_t *cmap,
                          int ids) {
    const int f = blockIdx.x;
    for (int t = coffs[f] + (int)threadIdx.x; t < coffs[f + 1]; t += blockDim.x)
        cmap[(int64_t)f * npt + epoint[clist[t]]] = ids ? clist[t] : t;
}

// The second pass's active set (Optimizer.cc:791-826: an observation with
// chi2 > 5.991 (mono) / 7.815 (stereo), or behind the camera, leaves it), on
// the device: the host's rule on the device's chi2 and front flags
__global__ void k_ba_pass2_active(const EdgeD *edges, int ne, const double *chi2, const uint8_t *front,
                                  uint8_t *active) {
    const int e = blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= ne) return;
    const double th = edges[e].stereo ? 7.815 : 5.991;
    active[e] = !(chi2[e] > th || !front[e]);
}

// Fast mode's active set on the device (a graph whose free cameras observe
// each point at most once): usable = active with a free camera, and the
// camera x point -> edge map the dense Schur product reads -- no host lists
__global__ void k_ba_usable_map(const uint8_t *active, const int32_t *efree, const int32_t *epoint, int ne, int npt,
                                uint8_t *usable, int32_t *cmap) {
    const int e = blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= ne) return;
    const int f = efree[e];
    const bool us = active[e] && f >= 0;
    usable[e] = us;
    if (us) cmap[(int64_t)f * npt + epoint[e]] = e;
}

// offs[0..n] = exclusive scan of cnt[0..n) (one workgroup of 1024: a
// contiguous range per thread, then a scan of the 1024 range sums)
__global__ __launch_bounds__(1024) void k_ba_scan_counts(const int32_t *cnt, int n, int32_t *offs) {
    __shared__ int32_t wsum[16];
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const int per = (n + 1023) / 1024, b = min(tid * per, n), e = min(b + per, n);
    int32_t sum = 0;
    for (int i = b; i < e; ++i) sum += cnt[i];
    int32_t incl = sum;   // inclusive scan over the wave
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const int32_t v = __shfl_up(incl, d, 64);
        if (lane >= d) incl += v;
    }
    if (lane == 63) wsum[w] = incl;
    __syncthreads();
    int32_t base = 0;
    for (int k = 0; k < w; ++k) base += wsum[k];
    int32_t at = base + incl - sum;
    for (int i = b; i < e; ++i) {
        offs[i] = at;
        at += cnt[i];
    }
    if (tid == 1023) offs[n] = at;   // (the last thread's range ends at n)
}

// S_{i1 i2} (+ lambda I on the diagonal blocks) -= sum over the pair's shared
// points, in point order, of (B Dinv)_{i1} B_{i2}^T, in two passes:
//  k_ba_pair_terms: every (shared point, block entry) term of every pair,
//    thread per term (the 3-term dot product in the sequential order);
//  k_ba_pairs_sum: workgroup per pair, lane = block entry, subtracts its
//    terms in point order (ordered_colsum: LDS-staged, double-buffered).
// Only the subtractions are sequential, so the longest pair (a camera with
// itself: all its points) costs a chain of dependent adds, not of loads.
__global__ void k_ba_pair_terms(const int2 *mlist, int64_t nterms, const int32_t *total, const EdgeOut *eo,
                                const double *bdinv, double *terms) {
    const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (idx >= nterms || idx >= 36 * (int64_t)*total) return;   // (launched over a bound; total: the lists' length)
    const int64_t t = idx / 36;
    const int e = (int)(idx - t * 36), r = e / 6, c = e % 6;
    const int2 mt = mlist[t];
    const double *bd = bdinv + 18 * (int64_t)mt.x + 3 * r;
    const double *hp = eo[mt.y].hpl + 3 * c;
    double sj = 0;
    for (int k = 0; k < 3; ++k) sj = sj + bd[k] * hp[k];
    terms[idx] = sj;
}

// Ordered sums per vertex, out[v][f] = sum over t in [offs[v], offs[v+1]) of
// rec[list[t]][field f] in list order (edges with pred[e] == 0 add nothing),
// in two passes:
//  k_ba_gather_rows: thread per (list entry, field) copies the records into
//    list order (+0.0 for a skipped edge: the running sum starts at +0.0 and
//    never becomes -0.0 under round-to-nearest, so adding +0.0 leaves it as it
//    is);
//  k_ba_stream_sums: workgroup per vertex, lane = field, adds its column in
//    list order (ordered_colsum) -- a chain of dependent adds, no dependent
//    loads.
// minus != nullptr: out = minus - sum (the reduced right-hand side).
// NF fields per record; LAYOUT 1: EdgeOut's hpp (36) then bp (6), 0: record
// fields 0..NF-1.
template <int NF, int LAYOUT>
__global__ void k_ba_gather_rows(const double *rec, int stride, const int32_t *list, int n, const uint8_t *pred,
                                 double *out, const int *gate) {
    if (gate && !*gate) return;
    const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (idx >= (int64_t)n * NF) return;
    const int t = (int)(idx / NF), f = (int)(idx - (int64_t)t * NF);
    const int e = list[t];
    const int off = LAYOUT == 1 && f >= 36 ? 63 + (f - 36) : f;   // EdgeOut::bp at 63
    out[idx] = (pred && !pred[e]) ? 0.0 : rec[(int64_t)e * stride + off];
}

// The ordered column sums of one vertex's rows (contiguous: nrows x NF
// doubles at base), acc_f = init_f (+|-) row_0[f] (+|-) row_1[f] ... in row
// order, in lane f < NF of wave 0.  One workgroup of kSumThreads per vertex
// streams the rows through two LDS buffers of kSumElems: every thread loads
// its share of chunk k + 1 into registers, wave 0 adds chunk k from LDS, then
// the registers go to the other buffer -- the chain of dependent adds runs
// while the next chunk is in flight (a wave alone kept too few loads in flight
// to cover the latency).
constexpr int kSumThreads = 1024, kSumElems = 8192, kSumPer = kSumElems / kSumThreads;
constexpr size_t kSumLds = 2 * kSumElems * sizeof(double);
template <int NF, bool SUB>
__device__ double ordered_colsum(const double *base, int nrows, double acc, double *buf) {
    constexpr int kAhead = 16;   // LDS reads in flight ahead of the adds (8 left the chain waiting on them)
    constexpr int kRows = kSumElems / NF, kE = kRows * NF;   // whole rows per chunk
    const int tid = threadIdx.x, total = nrows * NF, nch = (nrows + kRows - 1) / kRows;
    double r[kSumPer];
    auto fetch = [&](int k) {
#pragma unroll
        for (int j = 0; j < kSumPer; ++j) {
            const int i = tid + j * kSumThreads;
            r[j] = (i < kE && k * kE + i < total) ? base[(int64_t)k * kE + i] : 0.0;
        }
    };
    auto put = [&](int k) {
        double *d = buf + (k & 1) * kSumElems;
#pragma unroll
        for (int j = 0; j < kSumPer; ++j) {
            const int i = tid + j * kSumThreads;
            if (i < kE) d[i] = r[j];
        }
    };
    if (nch) {
        fetch(0);
        put(0);
    }
    __syncthreads();
    for (int k = 0; k < nch; ++k) {
        if (k + 1 < nch) fetch(k + 1);
        if (tid < NF) {
            const double *src = buf + (k & 1) * kSumElems + tid;
            const int nr = min(kRows, nrows - k * kRows);
            int q = 0;
            if (nr >= kAhead) {   // the reads of the next kAhead rows go out before this group's adds
                double a[kAhead];
#pragma unroll
                for (int u = 0; u < kAhead; ++u) a[u] = src[u * NF];
                for (; q + 2 * kAhead <= nr; q += kAhead) {
                    double b[kAhead];
#pragma unroll
                    for (int u = 0; u < kAhead; ++u) b[u] = src[(q + kAhead + u) * NF];
#pragma unroll
                    for (int u = 0; u < kAhead; ++u) acc = SUB ? acc - a[u] : acc + a[u];
#pragma unroll
                    for (int u = 0; u < kAhead; ++u) a[u] = b[u];
                }
#pragma unroll
                for (int u = 0; u < kAhead; ++u) acc = SUB ? acc - a[u] : acc + a[u];
                q += kAhead;
            }
            for (; q < nr; ++q) acc = SUB ? acc - src[q * NF] : acc + src[q * NF];
        }
        if (k + 1 < nch) put(k + 1);
        __syncthreads();
    }
    return acc;
}

// The fast mode's column sums (orbx_local_ba_fast): thread t adds field
// t % NF of rows t / NF, t / NF + G, ... (G = kSumThreads / NF groups; the
// loads coalesced, each thread's chain nrows / G long), then lane f < NF adds
// the G partial sums.  Same terms, another order: equal to rounding.
template <int NF, bool SUB>
__device__ double tree_colsum(const double *base, int nrows, double acc, double *buf) {
    constexpr int G = kSumThreads / NF;
    const int tid = threadIdx.x, f = tid % NF, g = tid / NF;
    double part = 0.0;
    if (g < G) {
        const double *src = base + f;
        int r = g;
        for (; r + 3 * G < nrows; r += 4 * G) {   // four rows in flight per thread
            const double a0 = src[(int64_t)r * NF], a1 = src[(int64_t)(r + G) * NF], a2 = src[(int64_t)(r + 2 * G) * NF],
                         a3 = src[(int64_t)(r + 3 * G) * NF];
            part += (a0 + a1) + (a2 + a3);
        }
        for (; r < nrows; r += G) part += src[(int64_t)r * NF];
        buf[g * NF + f] = part;
    }
    __syncthreads();
    if (tid < NF) {
        double s = 0.0;
        for (int k = 0; k < G; ++k) s += buf[k * NF + tid];
        acc = SUB ? acc - s : acc + s;
    }
    __syncthreads();
    return acc;
}

// S_{i1 i2} (+ lambda I on the diagonal blocks) - the pair's terms in point
// order, written with its mirror (the solver reads the full matrix)
template <bool FAST>
__global__ __launch_bounds__(kSumThreads) void k_ba_pairs_sum(const int2 *pairs, const int32_t *moffs,
                                                              const double *terms, const double *Hpp, double lambda,
                                                              int nf, double *S) {
    extern __shared__ double sbuf[];
    const int pi = blockIdx.x, lane = threadIdx.x;
    const int i1 = pairs[pi].x, i2 = pairs[pi].y, r = lane / 6, c = lane % 6;
    double acc = 0;
    if (i1 == i2 && lane < 36) {
        acc = Hpp[36 * (int64_t)i1 + lane];
        if (r == c) acc = acc + lambda;
    }
    const int t0 = moffs[pi];
    if constexpr (FAST) acc = tree_colsum<36, true>(terms + 36 * (int64_t)t0, moffs[pi + 1] - t0, acc, sbuf);
    else acc = ordered_colsum<36, true>(terms + 36 * (int64_t)t0, moffs[pi + 1] - t0, acc, sbuf);
    if (lane >= 36) return;
    const int n = 6 * nf;
    S[(int64_t)(6 * i1 + r) * n + 6 * i2 + c] = acc;
    S[(int64_t)(6 * i2 + c) * n + 6 * i1 + r] = acc;
}

typedef double orbx_f64x4 __attribute__((ext_vector_type(4)));

// Fast mode's Schur complement and reduced right-hand side as one dense
// product on the FP64 matrix cores (round 6; each (camera, point) observed at
// most once, use_map).  With D_p = Hll_p + lambda I = L_p L_p^T (k_ba_point's
// lu: L_p^-1 and u_p = L_p^-1 bl_p), S = Hpp + lambda I - sum_p B_p D_p^-1 B_p^T
// = Hpp + lambda I - W^T W and bs = bp - W^T u, with W's row 3p + k the k-th
// row of L_p^-1 B_p^T (6 columns per free camera).  One K x CT operand M holds
// W (columns [0, 16 TCe)), u (column 16 TCe) and zeros, K = 3 npt padded to
// whole chunks of kSchurKC rows; M^T M's needed 16x16 tiles -- S's lower
// triangle and the u column -- go in 2x2 tile blocks (a workgroup of four
// waves per (block, chunk), each wave a quarter of the chunk, four
// independent accumulators), the chunk partials summed in chunk order
// (deterministic).  It replaces the shared-point lists, the per-pair sums and
// the per-edge B D^-1 products; equal to rounding.
constexpr int kSchurKC = 512;
__global__ void k_ba_schur_ops(int npt, int nf, int CT, int ucol, int kp, const int32_t *cmap, const EdgeOut *eo,
                               int ne, const double *lu, double *M) {
    const int64_t idx = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
    if (idx >= (int64_t)kp * CT) return;
    const int k = (int)(idx / CT), col = (int)(idx - (int64_t)k * CT);
    const int p = k / 3, kk = k - 3 * p;
    double v = 0.0;
    if (p < npt) {
        const double *l = lu + 9 * (int64_t)p;   // L^-1 as m00, m10, m11, m20, m21, m22; then u
        if (col < 6 * nf) {
            const int f = col / 6, r = col - 6 * f;
            const int ed = cmap[(int64_t)f * npt + p];   // (the edge: k_ba_cmap / k_ba_usable_map with ids)
            if (ed >= 0 && ed < ne) {   // (-1: none; the bound guards the read whatever the map holds)
                const double *h = eo[ed].hpl + 3 * r;   // row r of B (6 x 3)
                v = kk == 0 ? l[0] * h[0]
                  : kk == 1 ? fma(l[2], h[1], l[1] * h[0])
                            : fma(l[5], h[2], fma(l[4], h[1], l[3] * h[0]));
            }
        } else if (col == ucol) {
            v = l[6 + kk];
        }
    }
    M[idx] = v;
}
__device__ inline void schur_block(int blk, int h, int &I0, int &J0) {   // 2x2 tile block -> its first tiles
    const int nl = h * (h + 1) / 2;
    int ip = 0, jp = blk;
    if (blk < nl) {
        while (jp > ip) { jp -= ip + 1; ++ip; }
    } else {
        ip = blk - nl;
        jp = h;
    }
    I0 = 2 * ip;
    J0 = 2 * jp;
}
__global__ __launch_bounds__(256) void k_ba_schur_mfma(const double *M, int CT, int h, double *part) {
    __shared__ double red[4][4 * 256];
    const int blk = blockIdx.x, ch = blockIdx.y, tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    int I0, J0;
    schur_block(blk, h, I0, J0);
    const int fr = lane & 15, fk = lane >> 4;
    const double *base = M + (int64_t)(ch * kSchurKC + w * (kSchurKC / 4) + fk) * CT + fr;
    const double *a0 = base + 16 * I0, *a1 = a0 + 16, *b0 = base + 16 * J0, *b1 = b0 + 16;
    orbx_f64x4 c00 = {0.0, 0.0, 0.0, 0.0}, c01 = c00, c10 = c00, c11 = c00;
    for (int s = 0; s < kSchurKC / 16; s += 4) {   // four K-steps' operands in flight
        double A0[4], A1[4], B0[4], B1[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const int64_t o = (int64_t)(4 * (s + u)) * CT;
            A0[u] = a0[o]; A1[u] = a1[o]; B0[u] = b0[o]; B1[u] = b1[o];
        }
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            c00 = __builtin_amdgcn_mfma_f64_16x16x4f64(A0[u], B0[u], c00, 0, 0, 0);
            c01 = __builtin_amdgcn_mfma_f64_16x16x4f64(A0[u], B1[u], c01, 0, 0, 0);
            c10 = __builtin_amdgcn_mfma_f64_16x16x4f64(A1[u], B0[u], c10, 0, 0, 0);
            c11 = __builtin_amdgcn_mfma_f64_16x16x4f64(A1[u], B1[u], c11, 0, 0, 0);
        }
    }
    // (tile q = 2 (I - I0) + (J - J0); element 4 lane + r: row (l >> 4) + 4 r, column l & 15)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
        red[w][0 * 256 + 4 * lane + r] = c00[r];
        red[w][1 * 256 + 4 * lane + r] = c01[r];
        red[w][2 * 256 + 4 * lane + r] = c10[r];
        red[w][3 * 256 + 4 * lane + r] = c11[r];
    }
    __syncthreads();
    double *o = part + ((int64_t)ch * gridDim.x + blk) * 1024;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        const int e = tid + 256 * q;
        o[e] = ((red[0][e] + red[1][e]) + red[2][e]) + red[3][e];
    }
}
// S's lower triangle = Hpp (+ lambda) on the diagonal blocks - (W^T W), and
// bs = bp - W^T u, the chunk partials added in chunk order
__global__ void k_ba_schur_sum(const double *part, int nch, int nblk, int h, const double *Hpp, const double *bp,
                               double lambda, int n, double *S, double *bs) {
    const int idx = blockIdx.x * blockDim.x + threadIdx.x;
    if (idx >= n * n + n) return;
    int row, col;
    if (idx < n * n) {
        row = idx / n;
        col = idx - row * n;
        if (col > row) return;
    } else {
        row = idx - n * n;
        col = -1;
    }
    const int I = row >> 4, ri = row & 15;
    int blk, q, cj;
    if (col >= 0) {
        const int J = col >> 4;
        blk = (I >> 1) * ((I >> 1) + 1) / 2 + (J >> 1);
        q = 2 * (I & 1) + (J & 1);
        cj = col & 15;
    } else {
        blk = h * (h + 1) / 2 + (I >> 1);
        q = 2 * (I & 1);
        cj = 0;
    }
    const int64_t off = 256 * q + 4 * (16 * (ri & 3) + cj) + (ri >> 2);
    double sum = 0.0;
    int c = 0;
    for (; c + 4 <= nch; c += 4) {   // (four independent loads, added in chunk order)
        const double v0 = part[((int64_t)c * nblk + blk) * 1024 + off], v1 = part[((int64_t)(c + 1) * nblk + blk) * 1024 + off],
                     v2 = part[((int64_t)(c + 2) * nblk + blk) * 1024 + off], v3 = part[((int64_t)(c + 3) * nblk + blk) * 1024 + off];
        sum = (((sum + v0) + v1) + v2) + v3;
    }
    for (; c < nch; ++c) sum += part[((int64_t)c * nblk + blk) * 1024 + off];
    if (col < 0) {
        bs[row] = bp[row] - sum;
        return;
    }
    const int i = row / 6, j = col / 6;
    double acc = 0.0;
    if (i == j) {
        acc = Hpp[36 * (int64_t)i + 6 * (row - 6 * i) + (col - 6 * j)];
        if (row == col) acc = acc + lambda;
    }
    S[idx] = acc - sum;
}

// out[v] = (minus[v] -) the ordered sum of the vertex's rows; fields [0, na)
// to out_a, the rest to out_b
template <int NF, bool FAST>
__global__ __launch_bounds__(kSumThreads) void k_ba_stream_sums(const double *rows, const int32_t *offs,
                                                                const double *minus, double *out_a, int na,
                                                                double *out_b, const int *gate) {
    if (gate && !*gate) return;   // (uniform: before any barrier)
    extern __shared__ double sbuf[];
    const int v = blockIdx.x, lane = threadIdx.x;
    const int t0 = offs[v];
    const double acc = FAST ? tree_colsum<NF, false>(rows + NF * (int64_t)t0, offs[v + 1] - t0, 0.0, sbuf)
                            : ordered_colsum<NF, false>(rows + NF * (int64_t)t0, offs[v + 1] - t0, 0.0, sbuf);
    if (lane >= NF) return;
    if (lane < na) out_a[(int64_t)v * na + lane] = minus ? minus[(int64_t)v * na + lane] - acc : acc;
    else out_b[(int64_t)v * (NF - na) + lane - na] = acc;
}

// (the ordered-sum kernels take 128 KB of LDS: raised once per kernel)
template <typename K>
bool sum_lds(K kernel) {
    return hipFuncSetAttribute(reinterpret_cast<const void *>(kernel), hipFuncAttributeMaxDynamicSharedMemorySize,
                               (int)kSumLds) == hipSuccess;
}
bool sums_ready() {
    static const bool ok = sum_lds(k_ba_pairs_sum<false>) && sum_lds(k_ba_stream_sums<6, false>) &&
                           sum_lds(k_ba_stream_sums<42, false>) && sum_lds(k_ba_pairs_sum<true>) &&
                           sum_lds(k_ba_stream_sums<6, true>) && sum_lds(k_ba_stream_sums<42, true>);
    return ok;
}

// Fast mode's trial readback, reduced on the device (parallel sums: equal to
// the host's ordered sums to rounding): out[0] = sum of rho0 over the active
// edges (activeRobustChi2); with x: out[1] = x (lambda x + b), poses then
// points (computeScale); out[2] = the solve flag; with Hpp: out[3] = the
// largest |diagonal| of the free vertices (computeLambdaInit).  kFastSumBlocks
// workgroups write partials; the last to finish (a counter it resets) folds
// them in a fixed order (lanes over blocks, then a butterfly), so the result
// does not depend on the schedule.
constexpr int kFastSumThreads = 256, kFastSumBlocks = 64;
__global__ __launch_bounds__(kFastSumThreads) void k_ba_fast_sums(const double *rho0, const uint8_t *active, int ne,
                                                                  const double *x, const double *bp, const double *bl,
                                                                  int n, int m, double lambda, const int *ok,
                                                                  const double *Hpp, int nf, const double *Hll, int np,
                                                                  double *part, unsigned *counter, double *out,
                                                                  double cur_chi, int *accept) {
    __shared__ double red[3][kFastSumThreads / 64];
    __shared__ bool last;
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const int gt = blockIdx.x * kFastSumThreads + tid, gs = gridDim.x * kFastSumThreads;
    double chi = 0, sc = 0, mx = 0;
    if (rho0)
        for (int e = gt; e < ne; e += gs)
            if (active[e]) chi += rho0[e];
    if (x && (!ok || *ok))
        for (int j = gt; j < m; j += gs) {
            const double xj = x[j];
            sc += xj * (lambda * xj + (j < n ? bp[j] : bl[j - n]));
        }
    if (Hpp) {
        for (int q = gt; q < 6 * nf; q += gs) mx = fmax(mx, fabs(Hpp[36 * (q / 6) + 7 * (q % 6)]));
        for (int q = gt; q < 3 * np; q += gs) mx = fmax(mx, fabs(Hll[9 * (q / 3) + 4 * (q % 3)]));
    }
    for (int o = 32; o > 0; o >>= 1) {
        chi += __shfl_xor(chi, o);
        sc += __shfl_xor(sc, o);
        mx = fmax(mx, __shfl_xor(mx, o));
    }
    if (lane == 0) { red[0][w] = chi; red[1][w] = sc; red[2][w] = mx; }
    __syncthreads();
    if (tid == 0) {
        double c = 0, t = 0, d = 0;
        for (int k = 0; k < kFastSumThreads / 64; ++k) { c += red[0][k]; t += red[1][k]; d = fmax(d, red[2][k]); }
        part[3 * blockIdx.x] = c;
        part[3 * blockIdx.x + 1] = t;
        part[3 * blockIdx.x + 2] = d;
        __threadfence();
        last = atomicAdd(counter, 1u) == gridDim.x - 1;
    }
    __syncthreads();
    if (!last || w != 0) return;
    __threadfence();
    // the last workgroup's wave 0 folds the partials: lane k takes blocks k,
    // k + 64, ... in order, then a fixed butterfly (the result does not
    // depend on the schedule)
    double c = 0, t = 0, d = 0;
    for (int k = lane; k < (int)gridDim.x; k += 64) {
        c += __builtin_nontemporal_load(&part[3 * k]);
        t += __builtin_nontemporal_load(&part[3 * k + 1]);
        d = fmax(d, __builtin_nontemporal_load(&part[3 * k + 2]));
    }
    for (int o = 32; o > 0; o >>= 1) {
        c += __shfl_xor(c, o);
        t += __shfl_xor(t, o);
        d = fmax(d, __shfl_xor(d, o));
    }
    if (lane != 0) return;
    out[0] = c;
    out[1] = t;
    out[2] = ok ? (double)*ok : 1.0;
    out[3] = d;
    if (accept) {   // lm_optimize's acceptance of the trial, the host's arithmetic exactly
        const bool okv = !ok || *ok != 0;
        const double tempChi = okv ? c : DBL_MAX;
        double rho = cur_chi - tempChi, sc = okv ? t : 0.0;
        sc += 1e-3;
        rho /= sc;
        const int a = rho > 0 && __builtin_isfinite(tempChi);
        *accept = a;
        out[8] = a;   // (h_fsum[8]: the host checks its own decision against it)
    }
    *counter = 0;
}

// Fast mode's trial tail in one kernel (k_ba_errors gated on the solve,
// then k_ba_fast_sums' trial sums): thread per edge computes its error and
// adds its rho0 (active edges), threads over [0, m) add x (lambda x + b);
// each workgroup writes its two partials, the last one (a counter it
// resets) folds them in a fixed order and writes the sums, the solve flag
// and the acceptance (as k_ba_fast_sums does) to the pinned readback.
constexpr int kErrSumThreads = 256;
__global__ __launch_bounds__(kErrSumThreads) void k_ba_errors_sums(
    const Pose *poses, const double *pts, const EdgeD *edges, int ne, const uint8_t *active, int robust,
    double *err_out, double *chi2_out, double *rho_out, uint8_t *front_out, const int *ok, const double *x,
    const double *bp, const double *bl, int n, int m, double lambda, double *part, unsigned *counter, double *out,
    double cur_chi, int *accept) {
    __shared__ double red[2][kErrSumThreads / 64];
    __shared__ bool last;
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, i = blockIdx.x * kErrSumThreads + tid;
    const int gs = gridDim.x * kErrSumThreads;
    const bool okv = !ok || *ok != 0;
    double chi = 0.0, sc = 0.0;
    if (okv) {
        if (i < ne)
            chi = ba_edge_error(i, poses, pts, edges, active, robust, 0, err_out, chi2_out, rho_out, front_out, nullptr);
        for (int j = i; j < m; j += gs) {
            const double xj = x[j];
            sc += xj * (lambda * xj + (j < n ? bp[j] : bl[j - n]));
        }
    }
    for (int o = 32; o > 0; o >>= 1) {
        chi += __shfl_xor(chi, o);
        sc += __shfl_xor(sc, o);
    }
    if (lane == 0) { red[0][w] = chi; red[1][w] = sc; }
    __syncthreads();
    if (tid == 0) {
        double c = 0, t = 0;
        for (int k = 0; k < kErrSumThreads / 64; ++k) { c += red[0][k]; t += red[1][k]; }
        part[2 * blockIdx.x] = c;
        part[2 * blockIdx.x + 1] = t;
        __threadfence();
        last = atomicAdd(counter, 1u) == gridDim.x - 1;
    }
    __syncthreads();
    if (!last || w != 0) return;
    __threadfence();
    double c = 0, t = 0;
    for (int k = lane; k < (int)gridDim.x; k += 64) {
        c += __builtin_nontemporal_load(&part[2 * k]);
        t += __builtin_nontemporal_load(&part[2 * k + 1]);
    }
    for (int o = 32; o > 0; o >>= 1) {
        c += __shfl_xor(c, o);
        t += __shfl_xor(t, o);
    }
    if (lane != 0) return;
    out[0] = c;
    out[1] = t;
    out[2] = ok ? (double)*ok : 1.0;
    const double tempChi = okv ? c : DBL_MAX;
    double rho = cur_chi - tempChi, s2 = okv ? t : 0.0;
    s2 += 1e-3;
    rho /= s2;
    const int a = rho > 0 && __builtin_isfinite(tempChi);
    if (accept) *accept = a;
    out[8] = a;
    *counter = 0;
}

__global__ void k_ba_restore(Pose *poses, int ncam, double *pts, int npt, const Pose *pose_bk, const double *pts_bk) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < ncam) poses[i] = pose_bk[i];
    if (i < npt)
        for (int k = 0; k < 3; ++k) pts[3 * (int64_t)i + k] = pts_bk[3 * (int64_t)i + k];
}

// Dense Cholesky S = L L^T (lower, in place, column by column) and the two
// triangular solves for x; one workgroup.  ok = 0 if S is not positive definite.
__global__ __launch_bounds__(1024) void k_ba_chol(double *S, int n, const double *bs, double *x, int *ok) {
    __shared__ double diag;
    __shared__ int bad;
    const int tid = threadIdx.x;
    if (tid == 0) bad = 0;
    __syncthreads();
    for (int j = 0; j < n; ++j) {
        if (tid == 0) {
            double d = S[(int64_t)j * n + j];
            for (int k = 0; k < j; ++k) d = d - S[(int64_t)j * n + k] * S[(int64_t)j * n + k];
            if (!(d > 0)) bad = 1;
            diag = sqrt(d);
            S[(int64_t)j * n + j] = diag;
        }
        __syncthreads();
        if (bad) break;
        for (int i = j + 1 + tid; i < n; i += blockDim.x) {
            double s = S[(int64_t)i * n + j];
            for (int k = 0; k < j; ++k) s = s - S[(int64_t)i * n + k] * S[(int64_t)j * n + k];
            S[(int64_t)i * n + j] = s / diag;
        }
        __syncthreads();
    }
    if (tid == 0) {
        *ok = !bad;
        if (!bad) {
            for (int i = 0; i < n; ++i) {   // L y = b
                double s = bs[i];
                for (int k = 0; k < i; ++k) s = s - S[(int64_t)i * n + k] * x[k];
                x[i] = s / S[(int64_t)i * n + i];
            }
            for (int i = n - 1; i >= 0; --i) {   // L^T x = y
                double s = x[i];
                for (int k = n - 1; k > i; --k) s = s - S[(int64_t)k * n + i] * x[k];
                x[i] = s / S[(int64_t)i * n + i];
            }
        }
    }
}

__device__ inline double readlane_f64(double v, int l) {
    const uint64_t u = __builtin_bit_cast(uint64_t, v);
    const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)u, l);
    const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(u >> 32), l);
    return __builtin_bit_cast(double, ((uint64_t)hi << 32) | lo);
}

// The same factorisation and solves with S held in LDS (n <= kCholLds),
// blocked right-looking in panels of kPanel columns:
//  - wave 0 factors a panel alone (lane t owns rows k+1+t and k+65+t of each
//    column k: scale by the diagonal, then the panel's own later columns get
//    their term L(i,k) L(j,k)); no workgroup barrier inside a panel;
//  - then all waves apply the panel to the trailing lower triangle, each entry
//    receiving the panel's kPanel terms one by one in ascending column.
//    Look-ahead: the next panel's columns get the terms first (all waves),
//    then wave 0 factors the next panel while waves 1.. update the rest, and
//    the last wave also runs the panel's forward-solve steps.
// Every entry therefore receives its terms L(i,m) L(j,m) in ascending m, each
// as its own multiply and subtract, exactly as the column-by-column factor
// (the oracle's): bit-identical, with two barriers per panel instead of one
// per column.  L stays in the lower triangle (row stride n+1: odd, so column
// reads spread over banks), the diagonal also in dg[].
//  - the solves run column-sweep in one wave (lane r owns rows r and r+64),
//    the backward one after the factor:
//    the forward terms arrive in ascending k as in the row loop, the
//    backward terms in descending k (the order the oracle uses).
constexpr int kCholLds = 128;
constexpr int kPanel = 8;
__global__ __launch_bounds__(512) void k_ba_chol_lds(const double *S, int n, const double *bs, double *x, int *ok,
                                                     unsigned long long *clk) {
    extern __shared__ double L[];   // n rows of n+1, then dg (n)
    __shared__ int bad;
    // clk (diagnostics, ORBX_BA_CLOCKS): wave 0's cycles in load / panel factor / next-panel update, then the backward solve
    unsigned long long c_t = clk ? __builtin_amdgcn_s_memtime() : 0, c_f = 0, c_u = 0, c_f2 = 0;
    const int ld = n + 1;
    double *dg = L + n * ld;
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, nw = blockDim.x >> 6;
    {   // the lower triangle, 8 loads in flight per thread
        const int tot = n * (n + 1) / 2;
        for (int q0 = tid; q0 < tot; q0 += 512 * 8) {
            double v[8];
            int at[8];
#pragma unroll
            for (int u = 0; u < 8; ++u) {
                const int q = q0 + 512 * u;
                at[u] = -1;
                if (q < tot) {
                    const int r = (int)((sqrt(8.0 * q + 1.0) - 1.0) * 0.5);   // row of packed index q
                    const int rr = r + (q >= (r + 1) * (r + 2) / 2) - (q < r * (r + 1) / 2);
                    const int c = q - rr * (rr + 1) / 2;
                    v[u] = S[(int64_t)rr * n + c];
                    at[u] = rr * ld + c;
                }
            }
#pragma unroll
            for (int u = 0; u < 8; ++u)
                if (at[u] >= 0) L[at[u]] = v[u];
        }
    }
    if (tid == 0) bad = 0;
    __syncthreads();
    if (clk && tid == 0) { clk[0] += __builtin_amdgcn_s_memtime() - c_t; c_t = __builtin_amdgcn_s_memtime(); }
    // wave 0 factors the panel [k0, k0 + kPanel): lane owns rows k0 + lane and
    // k0 + 64 + lane, the panel's columns of those rows in registers
    auto factor = [&](int k0) {
        const int k1 = min(k0 + kPanel, n);
        const int q0 = k0 + lane, q1 = k0 + 64 + lane;
        double p0[kPanel], p1[kPanel];
#pragma unroll
        for (int m = 0; m < kPanel; ++m) {
            p0[m] = (q0 < n && k0 + m < k1 && k0 + m <= q0) ? L[q0 * ld + k0 + m] : 0.0;
            p1[m] = (q1 < n && k0 + m < k1) ? L[q1 * ld + k0 + m] : 0.0;
        }
        // branch-free over the panel so the compiler can overlap column m's
        // tail with column m + 1's chain: a column past k1 (last panel only)
        // is all zeros with diagonal 1, so its terms subtract +0 (no-ops)
        bool good = true;
        double gl = 1.0;
#pragma unroll
        for (int m = 0; m < kPanel; ++m) {
            const int k = k0 + m;
            const double d = readlane_f64(p0[m], m);   // row k's diagonal entry (lane m)
            good = good && (k >= k1 || d > 0);
            const double g = sqrt(k < k1 ? d : 1.0);
            gl = lane == m ? g : gl;
            // column k below the diagonal: rows > k of this lane
            const double c0 = p0[m] / g;
            p0[m] = q0 > k ? c0 : p0[m];
            p1[m] = p1[m] / g;   // (q1 > k always)
#pragma unroll
            for (int jm = m + 1; jm < kPanel; ++jm) {   // the panel's later columns
                const double aj = readlane_f64(p0[m], jm);   // L(k0 + jm, k): row k0 + jm is lane jm's q0
                const double u0 = p0[jm] - p0[m] * aj;
                p0[jm] = q0 >= k0 + jm ? u0 : p0[jm];
                p1[jm] = p1[jm] - p1[m] * aj;
            }
        }
        if (!good && lane == 0) bad = 1;
        if (lane < k1 - k0) dg[k0 + lane] = gl;
#pragma unroll
        for (int m = 0; m < kPanel; ++m) {
            if (k0 + m >= k1) break;
            if (q0 < n && q0 > k0 + m) L[q0 * ld + k0 + m] = p0[m];
            if (q1 < n) L[q1 * ld + k0 + m] = p1[m];
        }
    };
    // the panel [k0, k1)'s terms for rows i .. i+3, columns [c0, row]: four
    // independent chains per lane sharing the column's panel values
    auto trail = [&](int i, int k0, int k1, int c0) {
        double li[4][kPanel];
#pragma unroll
        for (int r = 0; r < 4; ++r)
#pragma unroll
            for (int m = 0; m < kPanel; ++m) li[r][m] = (i + r < n && k0 + m < k1) ? L[(i + r) * ld + k0 + m] : 0.0;
        const int ie = min(i + 3, n - 1);
        for (int j = c0 + lane; j <= ie; j += 64) {
            double lj[kPanel], v[4];
#pragma unroll
            for (int m = 0; m < kPanel; ++m) lj[m] = k0 + m < k1 ? L[j * ld + k0 + m] : 0.0;
#pragma unroll
            for (int r = 0; r < 4; ++r) v[r] = (j <= i + r && i + r < n) ? L[(i + r) * ld + j] : 0.0;
#pragma unroll
            for (int m = 0; m < kPanel; ++m)
                if (k0 + m < k1) {
#pragma unroll
                    for (int r = 0; r < 4; ++r) v[r] = v[r] - li[r][m] * lj[m];
                }
#pragma unroll
            for (int r = 0; r < 4; ++r)
                if (j <= i + r && i + r < n) L[(i + r) * ld + j] = v[r];
        }
    };
    // the forward solve L y = b rides along in wave ws: panel [k0, k1)'s
    // steps run while wave 0 factors the next panel (lane r owns rows r and
    // r + 64; each s_i receives its terms in ascending k, as in the row loop)
    const int ws = nw / 2, i0 = lane, i1 = lane + 64, r0 = min(i0, n - 1), r1 = min(i1, n - 1);
    double s0 = 0.0, s1 = 0.0;
    if (w == ws) {
        s0 = i0 < n ? bs[i0] : 0.0;
        s1 = i1 < n ? bs[i1] : 0.0;
    }
    auto forward = [&](int k0, int k1) {
        double a0[kPanel], a1[kPanel], dk[kPanel];
#pragma unroll
        for (int m = 0; m < kPanel; ++m) {
            const int kk = min(k0 + m, n - 1);
            dk[m] = dg[kk];
            a0[m] = L[r0 * ld + kk];
            a1[m] = L[r1 * ld + kk];
        }
#pragma unroll
        for (int m = 0; m < kPanel; ++m) {
            const int k = k0 + m;
            if (k >= k1) break;
            const double yk = (k < 64 ? readlane_f64(s0, k) : readlane_f64(s1, k - 64)) / dk[m];
            if (lane == (k & 63)) (k < 64 ? s0 : s1) = yk;
            if (i0 > k && i0 < n) s0 = s0 - a0[m] * yk;
            if (i1 > k && i1 < n) s1 = s1 - a1[m] * yk;
        }
    };
    // look-ahead: while wave 0 factors panel p + 1, the other waves apply panel
    // p to the columns past it (the next panel's columns got panel p's terms
    // first, from every wave)
    if (w == 0) factor(0);
    __syncthreads();
    if (clk && tid == 0) { const unsigned long long t = __builtin_amdgcn_s_memtime(); c_f += t - c_t; c_t = t; }
    for (int k0 = 0; k0 < n && !bad; k0 += kPanel) {
        const int k1 = min(k0 + kPanel, n), k2 = min(k1 + kPanel, n), pw = k2 - k1;
        for (int e = tid; e < (n - k1) * pw; e += blockDim.x) {   // next panel's columns, rows >= k1
            const int i = k1 + e / pw, j = k1 + e % pw;
            if (j > i) continue;
            double v = L[i * ld + j];
#pragma unroll
            for (int m = 0; m < kPanel; ++m)
                if (k0 + m < k1) v = v - L[i * ld + k0 + m] * L[j * ld + k0 + m];
            L[i * ld + j] = v;
        }
        __syncthreads();
        if (clk && tid == 0) { const unsigned long long t = __builtin_amdgcn_s_memtime(); c_u += t - c_t; c_t = t; }
        const unsigned long long c_w = clk ? __builtin_amdgcn_s_memtime() : 0;
        if (w == 0) {
            if (k1 < n) factor(k1);
            if (clk && lane == 0) c_f2 += __builtin_amdgcn_s_memtime() - c_w;
        } else {
            if (w == ws) forward(k0, k1);
            else   // (waves other than 0 and ws)
                for (int i = k2 + 4 * (w - 1 - (w > ws)); i < n; i += 4 * (nw - 2)) trail(i, k0, k1, k2);
            if (clk && lane == 0) c_f2 += __builtin_amdgcn_s_memtime() - c_w;
        }
        __syncthreads();
        if (clk && tid == 0) { const unsigned long long t = __builtin_amdgcn_s_memtime(); c_f += t - c_t; c_t = t; }
    }
    if (clk && tid == 0) { clk[1] += c_f; clk[2] += c_u; }
    if (clk && lane == 0 && (w == 0 || w == 1 || w == ws)) atomicAdd(clk + (w == 0 ? 5 : w == 1 ? 6 : 7), c_f2);
    if (w != ws) return;
    if (clk) c_t = __builtin_amdgcn_s_memtime();
    const bool good = !bad;
    if (lane == 0) *ok = good;
    if (!good) return;
    double dk, a0, a1;
    dk = dg[n - 1];
    a0 = L[(n - 1) * ld + r0];
    a1 = L[(n - 1) * ld + r1];
    for (int k = n - 1; k >= 0; --k) {   // L^T x = y
        const int kn = max(k - 1, 0);
        const double dn = dg[kn], a0n = L[kn * ld + r0], a1n = L[kn * ld + r1];
        const double xk = (k < 64 ? readlane_f64(s0, k) : readlane_f64(s1, k - 64)) / dk;
        if (lane == (k & 63)) (k < 64 ? s0 : s1) = xk;
        if (i0 < k) s0 = s0 - a0 * xk;
        if (i1 < k) s1 = s1 - a1 * xk;
        dk = dn; a0 = a0n; a1 = a1n;
    }
    if (i0 < n) x[i0] = s0;
    if (i1 < n) x[i1] = s1;
    if (clk && lane == 0) { clk[3] += __builtin_amdgcn_s_memtime() - c_t; clk[4] += 1; }
}

// Fast mode's factorisation (equal to rounding, not in the ordered mode's
// term order): the augmented matrix [S b; b^T .] = L L^T, so row n of L is
// y = L^-1 b and the forward solve comes free, right-looking in 16-column
// panels on the FP64 matrix cores, with the latency chain cut to what the
// panel needs:
//  - L in LDS (16T rows of ld, T = tile rows of the n + 1 rows), the
//    reciprocal diagonal in rinv[];
//  - the 16x16 tiles right of the first panel live in the accumulators of
//    waves 3..7 (tile t of the column-major lower-triangle order -> wave
//    3 + t % 5, slot t / 5), each receives panel J as four
//    v_mfma_f64_16x16x4 with A = -L(rows of I, J), B = L(rows of K, J)^T,
//    and goes to LDS once, when it is the next panel;
//  - waves 0..2 factor a panel, rows on the lanes: each holds the diagonal
//    block in lanes 0..15 and a third of the rows below in lanes 16..63, and
//    runs the same pivot chain -- a column's pivot by readlane, 1/sqrt as rsq
//    plus one Newton step, the column scaled by it; the next column gets its
//    term at once (readlane), the later ones a column later from an LDS
//    broadcast -- no division, square root or exchange between waves;
//  - look-ahead: the owners of the next panel's tiles apply the panel first
//    and store them, then waves 0..2 factor the next panel while the owners
//    apply the panel to everything else: two barriers a panel;
//  - L^T x = y column-sweep in wave 0 (x_k = s_k * rinv_k), 16 rows a block
//    with the block's coefficients loaded together and no branch per step.
// Measured (profiles/r06_ab_ba_chol_fast.txt, r06_ab_ba_chol_3w.txt): 85 ->
// 42 us a factorisation with wave 0 factoring alone, fast local BA 5.0 ->
// 4.2 ms on one box; then the three factor waves.
// ok = 0 if a pivot is not positive.  n <= kCholFastMax (n + 1 rows <= 128).
constexpr int kCholFastMax = 126;
__device__ inline double rsq_nr(double d) {   // 1/sqrt(d): the hardware estimate and one Newton step
    const double r = __builtin_amdgcn_rsq(d);
    const double h = 0.5 * d * r;
    return fma(r, fma(-r, h, 0.5), r);
}
__device__ inline int chol_tile(int t, int T, int TC) {   // tile t (K >= 1, column-major) -> (I << 8) | K, or -1
    for (int k = 1; k < TC; ++k) {
        if (t < T - k) return ((k + t) << 8) | k;
        t -= T - k;
    }
    return -1;
}
__global__ __launch_bounds__(512) void k_ba_chol_fast(const double *S, int n, const double *bs, double *x, int *ok,
                                                      unsigned long long *clk) {
    extern __shared__ double L[];   // 16T rows of ld, rinv (16T), the factor waves' column broadcasts (3 x 16 x 64)
    __shared__ int bad;
    constexpr int kSlots = 6;   // (T <= 8: at most 28 tiles right of the first panel, 6 a wave over waves 3..7)
    const int T = (n + 16) / 16, TC = (n + 15) / 16, R = 16 * T, ld = R + 1;
    double *rinv = L + R * ld;
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    // clk (diagnostics, ORBX_BA_CLOCKS): wave 0's cycles in load / factor / waits / backward solve
    unsigned long long c_t = clk ? __builtin_amdgcn_s_memtime() : 0, c_f = 0;
    // load: rows 0..n-1 of S's lower triangle, row n = b, zeros elsewhere
    // (a wave's 16 rows: all 32 loads in flight, then the stores)
    {
        double v[16][2];
#pragma unroll
        for (int i = 0; i < 16; ++i) {
            const int r = w + 8 * i;
#pragma unroll
            for (int h = 0; h < 2; ++h) {
                const int c = lane + 64 * h;
                v[i][h] = r < n ? (c <= r ? S[(int64_t)r * n + c] : 0.0) : (r == n && c < n ? bs[c] : 0.0);
            }
        }
#pragma unroll
        for (int i = 0; i < 16; ++i)
#pragma unroll
            for (int h = 0; h < 2; ++h)
                if (w + 8 * i < R && lane + 64 * h < R) L[(w + 8 * i) * ld + lane + 64 * h] = v[i][h];
    }
    if (tid == 0) bad = 0;
    __syncthreads();
    if (clk && tid == 0) { clk[0] += __builtin_amdgcn_s_memtime() - c_t; c_t = __builtin_amdgcn_s_memtime(); }
    // Waves 0..2 factor a panel together, each on its own rows and with no
    // exchange: lanes 0..15 hold the panel's diagonal block (the same rows in
    // all three, so each wave runs the same pivot chain), lanes 16..63 of wave
    // f the rows k0 + 48 f + lane below it -- a third of the row updates each.
    auto factor = [&](int J) {
        const int k0 = 16 * J, q = lane < 16 ? k0 + lane : k0 + 48 * w + lane;
        double p0[16];
#pragma unroll
        for (int m = 0; m < 16; ++m) p0[m] = q < R ? L[q * ld + k0 + m] : 0.0;
        // Column m's terms reach column m + 1 at once (a readlane: the next
        // pivot's chain) and columns m + 2.. one column later, from entries
        // published to LDS and read back broadcast while the next pivot is
        // worked out.  (Unpredicated: a lane's entries above the diagonal take
        // finite garbage that only flows into its own upper entries, which are
        // neither read back nor stored.)  Every lane publishes its entry (no
        // exec-masked store), into its wave's own 16 x 64 buffer.
        double *cb = rinv + R + 1024 * w;
        double c[16];
        bool good = true;
        double rl = 0.0;
#pragma unroll
        for (int m = 0; m < 16; ++m) {
            if (k0 + m >= n) break;   // (uniform: the padding columns stay zero)
            const double d = readlane_f64(p0[m], m);   // the pivot: row k0 + m is lane m's
            good = good && d > 0;
            const double r = rsq_nr(d);
            rl = lane == m ? r : rl;
            p0[m] = p0[m] * r;
            if (m + 1 < 16) {
                const double a = readlane_f64(p0[m], m + 1);
                p0[m + 1] = fma(-p0[m], a, p0[m + 1]);
            }
            double cn[16];
            if (m + 2 < 16) {
                cb[64 * m + lane] = p0[m];
#pragma unroll
                for (int jm = m + 2; jm < 16; ++jm) cn[jm] = cb[64 * m + jm];
            }
            if (m >= 1)
#pragma unroll
                for (int jm = m + 1; jm < 16; ++jm) p0[jm] = fma(-p0[m - 1], c[jm], p0[jm]);   // column m - 1's terms
#pragma unroll
            for (int jm = m + 2; jm < 16; ++jm) c[jm] = cn[jm];
        }
        if (w == 0) {
            if (!good && lane == 0) bad = 1;
            if (lane < 16 && k0 + lane < n) rinv[k0 + lane] = rl;
        }
#pragma unroll
        for (int m = 0; m < 16; ++m) {
            if (k0 + m >= n) break;
            if (q < R && (lane < 16 ? w == 0 && q > k0 + m : true)) L[q * ld + k0 + m] = p0[m];
        }
    };
    // this wave's tiles and their accumulators (C[(l >> 4) + 4 r][l & 15] in element r)
    int tI[kSlots], tK[kSlots];
    orbx_f64x4 acc[kSlots];
    const int fr = lane & 15, fk = lane >> 4;   // fragment row / k of the MFMA operands
#pragma unroll
    for (int s = 0; s < kSlots; ++s) {
        const int tk = w >= 3 ? chol_tile(w - 3 + 5 * s, T, TC) : -1;
        tI[s] = tk >> 8;
        tK[s] = tk < 0 ? -1 : tk & 255;
        if (tK[s] >= 0)
#pragma unroll
            for (int r = 0; r < 4; ++r) acc[s][r] = L[(16 * tI[s] + fk + 4 * r) * ld + 16 * tK[s] + fr];
    }
    auto apply = [&](int s, int J) {   // panel J's terms into slot s
        orbx_f64x4 c = acc[s];
        const double *a = L + (16 * tI[s] + fr) * ld + 16 * J + fk, *b = L + (16 * tK[s] + fr) * ld + 16 * J + fk;
#pragma unroll
        for (int q = 0; q < 4; ++q) c = __builtin_amdgcn_mfma_f64_16x16x4f64(-a[4 * q], b[4 * q], c, 0, 0, 0);
        acc[s] = c;
    };
    if (w < 3) factor(0);
    if (clk && tid == 0) { const unsigned long long t = __builtin_amdgcn_s_memtime(); c_f += t - c_t; }
    __syncthreads();
    for (int J = 0; J + 1 < TC && !bad; ++J) {
#pragma unroll
        for (int s = 0; s < kSlots; ++s)
            if (tK[s] == J + 1) {   // the next panel's tiles: apply, store
                apply(s, J);
#pragma unroll
                for (int r = 0; r < 4; ++r) L[(16 * tI[s] + fk + 4 * r) * ld + 16 * tK[s] + fr] = acc[s][r];
            }
        __syncthreads();
        if (w < 3) {
            const unsigned long long c_w = clk ? __builtin_amdgcn_s_memtime() : 0;
            factor(J + 1);
            if (clk) c_f += __builtin_amdgcn_s_memtime() - c_w;
        } else {
#pragma unroll
            for (int s = 0; s < kSlots; ++s)
                if (tK[s] > J + 1) apply(s, J);
        }
        __syncthreads();
    }
    if (w != 0) return;
    if (clk && lane == 0) {
        const unsigned long long t = __builtin_amdgcn_s_memtime();
        clk[1] += t - c_t; clk[5] += c_f; c_t = t;
    }
    const bool good = !bad;
    if (lane == 0) *ok = good;
    if (!good) return;
    // L^T x = y: lane owns rows lane and lane + 64; y = row n of L
    const int i0 = lane, i1 = lane + 64, r0 = min(i0, n - 1), r1 = min(i1, n - 1);
    // 16 rows a block from the bottom: the block's coefficients (zero for
    // rows >= k) and reciprocals loaded together, then its steps from
    // registers -- a step on the chain is readlane, multiply, FMA; x_k is kept
    // aside
    double s0 = i0 < n ? L[n * ld + i0] : 0.0, s1 = i1 < n ? L[n * ld + i1] : 0.0, x0 = 0.0, x1 = 0.0;
    auto block = [&](int kb, auto hi_c) {   // rows kb..kb+15, all in one half (hi: rows 64..)
        constexpr bool hi = decltype(hi_c)::value;
        double a0[16], a1[16], rr[16];
#pragma unroll
        for (int u = 0; u < 16; ++u) {   // (a row past n - 1: r = 0, a no-op step)
            const int k = min(kb + u, n - 1);
            rr[u] = kb + u < n ? rinv[k] : 0.0;
            a0[u] = i0 < k ? L[k * ld + r0] : 0.0;
            a1[u] = i1 < k ? L[k * ld + r1] : 0.0;
        }
#pragma unroll
        for (int u = 15; u >= 0; --u) {
            const int k = kb + u;
            const double xk = readlane_f64(hi ? s1 : s0, hi ? k - 64 : k) * rr[u];
            if constexpr (hi) x1 = lane == k - 64 ? xk : x1;
            else x0 = lane == k ? xk : x0;
            s0 = fma(-a0[u], xk, s0);
            s1 = fma(-a1[u], xk, s1);
        }
    };
    for (int kb = (n - 1) & ~15; kb >= 0; kb -= 16) {   // (a block lies in one half: uniform branch per block)
        if (kb >= 64) block(kb, std::true_type{});
        else block(kb, std::false_type{});
    }
    if (i0 < n) x[i0] = x0;
    if (i1 < n) x[i1] = x1;
    if (clk && lane == 0) { clk[3] += __builtin_amdgcn_s_memtime() - c_t; clk[4] += 1; }
}

// the caller's edges as EdgeD (float -> double: exact) and the edge -> point list
__global__ void k_ba_edges(const orbx_ba_edge *in, int ne, double th_mono, double th_stereo, EdgeD *out,
                           int32_t *epoint) {
    const int e = blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= ne) return;
    const orbx_ba_edge s = in[e];
    EdgeD d;
    d.cam = s.cam; d.point = s.point; d.stereo = s.ur >= 0 ? 1 : 0; d.pad = 0;
    d.obs[0] = s.u; d.obs[1] = s.v; d.obs[2] = d.stereo ? s.ur : 0.0;
    d.omega = s.inv_sigma2;
    d.fx = s.fx; d.fy = s.fy; d.cx = s.cx; d.cy = s.cy; d.bf = s.bf;
    d.delta = d.stereo ? th_stereo : th_mono;
    out[e] = d;
    epoint[e] = s.point;
}

// xl = Dinv (bl - sum over the point's usable edges (camera order) of B^T xp)
// The back substitution in two passes:
//  k_ba_backsub_terms: thread per (point, edge) list entry: s = B^T (-xp) of a
//    usable edge (each component its own 6-term sum from 0), flagged;
//  k_ba_backsub: thread per point: cl = bl + the flagged terms in list order,
//    xl = Dinv cl -- the loads contiguous per point and off the add chain.
__global__ void k_ba_backsub_terms(int ne, const int32_t *list, const uint8_t *usable, const EdgeOut *eo,
                                   const EdgeD *edges, const Pose *poses, const double *xp, double *terms,
                                   uint8_t *flag) {
    const int t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= ne) return;
    const int ei = list[t];
    const bool u = usable[ei];
    flag[t] = u;
    if (!u) return;
    const int f = poses[edges[ei].cam].free_idx;
    const double *B = eo[ei].hpl;
    for (int c = 0; c < 3; ++c) {
        double a = 0;
        for (int r = 0; r < 6; ++r) a = a + B[3 * r + c] * -xp[6 * f + r];
        terms[3 * (int64_t)t + c] = a;
    }
}

__global__ void k_ba_backsub(const double *dinv, const double *bl, int npt, const int32_t *offs,
                             const double *terms, const uint8_t *flag, double *xl) {
    const int pt = blockIdx.x * blockDim.x + threadIdx.x;
    if (pt >= npt) return;
    double cl[3];
    for (int k = 0; k < 3; ++k) cl[k] = bl[3 * (int64_t)pt + k];
    const int te = offs[pt + 1];
    for (int t = offs[pt]; t < te; t += 4) {
        bool u[4];
        double s[4][3];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            u[j] = t + j < te && flag[t + j];
#pragma unroll
            for (int c = 0; c < 3; ++c) s[j][c] = u[j] ? terms[3 * (int64_t)(t + j) + c] : 0.0;
        }
#pragma unroll
        for (int j = 0; j < 4; ++j)
            if (u[j])
#pragma unroll
                for (int c = 0; c < 3; ++c) cl[c] = cl[c] + s[j][c];
    }
    const double *D = dinv + 9 * (int64_t)pt;
    for (int r = 0; r < 3; ++r) {
        double acc = 0;
        for (int c = 0; c < 3; ++c) acc = acc + D[3 * r + c] * cl[c];
        xl[3 * (int64_t)pt + r] = acc;
    }
}

// Fast mode's back substitution from the dense Schur operand (dense mode):
// xl_p = D_p^-1 (bl_p - sum_e B_e^T xc) = L_p^-T (u_p - (W xc)_p), W's rows
// 3p..3p+2 read once, a wave per point (lanes over the camera columns, a
// butterfly per row).  Replaces k_ba_backsub_terms + k_ba_backsub there.
__global__ __launch_bounds__(256) void k_ba_backsub_dense(const double *M, int CT, int ncols, const double *xc,
                                                          const double *lu, int npt, double *xl) {
    const int lane = threadIdx.x & 63, p = blockIdx.x * 4 + (threadIdx.x >> 6);
    if (p >= npt) return;
    const double *row = M + (int64_t)3 * p * CT;
    double r0 = 0.0, r1 = 0.0, r2 = 0.0;
    for (int c = lane; c < ncols; c += 64) {
        const double x = xc[c];
        r0 = fma(row[c], x, r0);
        r1 = fma(row[CT + c], x, r1);
        r2 = fma(row[2 * CT + c], x, r2);
    }
    for (int o = 32; o > 0; o >>= 1) {
        r0 += __shfl_xor(r0, o);
        r1 += __shfl_xor(r1, o);
        r2 += __shfl_xor(r2, o);
    }
    if (lane != 0) return;
    const double *l = lu + 9 * (int64_t)p;   // L^-1 (m00, m10, m11, m20, m21, m22), then u
    const double y0 = l[6] - r0, y1 = l[7] - r1, y2 = l[8] - r2;
    double *o = xl + 3 * (int64_t)p;   // L^-T y
    o[0] = l[0] * y0 + l[1] * y1 + l[3] * y2;
    o[1] = l[2] * y1 + l[4] * y2;
    o[2] = l[5] * y2;
}

// SE3Quat::exp(update) * estimate (se3quat.h:223-258, :104-110); points += dx
// bk (nullable): the estimate before the step is saved first (the trial's
// push(); a rejected trial that ran the step restores it with k_ba_restore)
__global__ void k_ba_update(Pose *poses, int ncam, double *pts, int npt, const double *xp, const double *xl,
                            const int *gate, Pose *pose_bk, double *pts_bk) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (gate && !*gate) return;
    if (pose_bk) {
        if (i < ncam) pose_bk[i] = poses[i];
        if (i < npt)
            for (int k = 0; k < 3; ++k) pts_bk[3 * (int64_t)i + k] = pts[3 * (int64_t)i + k];
    }
    if (i < npt)
        for (int k = 0; k < 3; ++k) pts[3 * (int64_t)i + k] = pts[3 * (int64_t)i + k] + xl[3 * (int64_t)i + k];
    if (i < ncam && poses[i].free_idx >= 0) {
        Pose &T = poses[i];
        const double *u = xp + 6 * T.free_idx;
        const double w[3] = {u[0], u[1], u[2]}, ups[3] = {u[3], u[4], u[5]};
        const double theta = sqrt(w[0] * w[0] + w[1] * w[1] + w[2] * w[2]);
        const double Om[9] = {0, -w[2], w[1], w[2], 0, -w[0], -w[1], w[0], 0};
        double O2[9];
        for (int r = 0; r < 3; ++r)
            for (int c = 0; c < 3; ++c) {
                double acc = 0;
                for (int k = 0; k < 3; ++k) acc = acc + Om[3 * r + k] * Om[3 * k + c];
                O2[3 * r + c] = acc;
            }
        double R[9], V[9];
        if (theta < 0.00001) {
            for (int k = 0; k < 9; ++k) R[k] = ((k % 4 == 0) ? 1.0 : 0.0) + Om[k] + O2[k];
            for (int k = 0; k < 9; ++k) V[k] = R[k];
        } else {
            const double a = sin(theta) / theta, b = (1 - cos(theta)) / (theta * theta);
            const double c = (theta - sin(theta)) / pow(theta, 3);
            for (int k = 0; k < 9; ++k) {
                R[k] = ((k % 4 == 0) ? 1.0 : 0.0) + a * Om[k] + b * O2[k];
                V[k] = ((k % 4 == 0) ? 1.0 : 0.0) + b * Om[k] + c * O2[k];
            }
        }
        double qe[4], te[3];
        R_to_quat(R, qe);
        for (int r = 0; r < 3; ++r) te[r] = V[3 * r] * ups[0] + V[3 * r + 1] * ups[1] + V[3 * r + 2] * ups[2];
        quat_normalize(qe);   // SE3Quat(q, t) constructor
        // (qe, te) * (T.q, T.t): t = te + qe * T.t, q = qe * T.q, normalised
        double rt[3], qn[4];
        quat_rotate(qe, T.t, rt);
        for (int k = 0; k < 3; ++k) T.t[k] = te[k] + rt[k];
        quat_mul(qe, T.q, qn);
        quat_normalize(qn);
        for (int k = 0; k < 4; ++k) T.q[k] = qn[k];
    }
}

}  // namespace
}  // namespace orbx

using namespace orbx;

namespace {

// Converter::toSE3Quat (Converter.cc:37-47): SE3Quat(R, t) from a float Tcw
void pose_from_cv(const float *T, Pose &p) {
    double R[9];
    for (int r = 0; r < 3; ++r)
        for (int c = 0; c < 3; ++c) R[3 * r + c] = T[4 * r + c];
    R_to_quat(R, p.q);
    quat_normalize(p.q);
    for (int r = 0; r < 3; ++r) p.t[r] = T[4 * r + 3];
}

// Converter::toCvMat(SE3Quat): rotation matrix and translation as float
void pose_to_cv(const Pose &p, float *T) {
    double R[9];
    quat_to_R(p.q, R);
    for (int r = 0; r < 3; ++r) {
        for (int c = 0; c < 3; ++c) T[4 * r + c] = (float)R[3 * r + c];
        T[4 * r + 3] = (float)p.t[r];
    }
}

struct Dev {
    uint8_t *base = nullptr;
    size_t cap = 0;
};

template <typename T>
T *carve(uint8_t *&p, size_t n) {
    T *r = reinterpret_cast<T *>(p);
    p += (sizeof(T) * n + 255) & ~size_t(255);
    return r;
}

struct Graph {
    int ncam, npt, ne, nf;
    std::vector<Pose> poses;
    const orbx_ba_edge *raw;   // the caller's edges (converted to EdgeD on the device)
    std::vector<int32_t> coffs, clist, poffs, plist, epoint;   // camera lists: usable edges by point; point lists: edges by camera
    std::vector<int32_t> efree;   // per edge: its camera's free index (-1: fixed), for the host's list building
};

// Per-device workspace kept across calls (LocalMapping runs a BA per
// keyframe): the stream, the device arena, the pinned readback buffers and
// the pair lists, grown on demand.  Allocating and freeing them per call cost
// ~5 ms of the ~15 ms a KITTI-size call took.
struct BAWs {
    std::mutex mu;
    hipStream_t st = nullptr;
    hipEvent_t ev = nullptr;   // (fast mode: the trial's readback, waited on while the speculative build runs)
    uint8_t *dev = nullptr, *host = nullptr;
    size_t cap = 0, hcap = 0;
    int32_t *moffs = nullptr;
    size_t moffs_cap = 0;
    int2 *mlist = nullptr;
    double *terms = nullptr;
    int64_t mcap = 0;
};

BAWs &ba_ws(int device) {
    static BAWs ws[64];
    return ws[device & 63];
}

template <typename T>
bool grow_dev(T *&p, size_t &cap, size_t need) {
    if (need <= cap && p) return true;
    if (p) (void)hipFree(p);
    p = nullptr;
    cap = 0;
    if (hipMalloc(reinterpret_cast<void **>(&p), sizeof(T) * need) != hipSuccess) return false;
    cap = need;
    return true;
}

// ORBX_BA_CLOCKS: k_ba_chol_lds / k_ba_chol_fast phase cycles, summed over the process and
// printed at exit (diagnostics)
unsigned long long *chol_clk() {
    static unsigned long long *p = nullptr;
    static bool init = false;
    if (!init) {
        init = true;
        if (std::getenv("ORBX_BA_CLOCKS") && hipMallocManaged(reinterpret_cast<void **>(&p), 64) == hipSuccess) {
            std::memset(p, 0, 64);
            std::atexit([] {
                (void)hipDeviceSynchronize();
                std::fprintf(stderr, "cholesky cycles per call (k_ba_chol_lds / k_ba_chol_fast): load %llu panel %llu trailing %llu solves %llu (%llu calls); factor %llu trail(w1) %llu fwd(ws) %llu\n",
                             p[0] / std::max(p[4], 1ull), p[1] / std::max(p[4], 1ull), p[2] / std::max(p[4], 1ull),
                             p[3] / std::max(p[4], 1ull), p[4], p[5] / std::max(p[4], 1ull), p[6] / std::max(p[4], 1ull),
                             p[7] / std::max(p[4], 1ull));
            });
        }
    }
    return p;
}

// ORBX_BA_CHOL_FAST=0: fast mode factors with the ordered mode's kernel;
// ORBX_BA_DENSE_SCHUR=0: fast mode's Schur pairs as shared-point lists + pair
// sums, as the ordered mode's (diagnostics, A/B)
bool env_on(const char *name) {
    const char *e = std::getenv(name);
    return !e || std::atoi(e) != 0;
}
bool chol_fast_on() {
    static const bool on = env_on("ORBX_BA_CHOL_FAST");
    return on;
}
bool dense_schur_on() {
    static const bool on = env_on("ORBX_BA_DENSE_SCHUR");
    return on;
}

class BA {
public:
    BA(Graph &g, BAWs &ws) : g_(g), st_(ws.st), ws_(ws) {}
    int alloc();
    int upload(const double *pts);
    void set_active(const std::vector<uint8_t> &act);
    int set_active_pass2();   // (fast mode, device-built sets) the second pass's set without a round trip
    int errors(bool robust, double *chi_sum);
    int build(const int *gate = nullptr);
    int solve(double lambda, int *ok);
    // the LM driver's asynchronous pieces: launches and readbacks into pinned
    // host buffers, one stream synchronisation per trial
    int errors_async(bool robust, const int *gate);
    int solve_async(double lambda);
    int update_gated();
    int read_errors();
    int read_diag();
    int read_trial(double lambda, double cur_chi);
    int errors_trial(bool robust, double lambda, double cur_chi);   // (fast mode) errors_async + read_trial in one kernel
    double chi_sum_host() const;
    double max_diag_host() const;
    double scale_host(double lambda) const;
    bool trial_ok() const { return fast_ ? h_fsum[2] != 0 : *h_ok != 0; }
    int pop();
    int download(double *pts, std::vector<double> &chi2, std::vector<uint8_t> &front);
    // (the buffers belong to the workspace)

    Graph &g_;
    hipStream_t st_;
    BAWs &ws_;
    bool fast_ = false;   // orbx_local_ba_fast: the per-vertex / per-pair sums as parallel reductions (equal to rounding)
    uint8_t *buf_ = nullptr;
    Pose *d_pose = nullptr, *d_pose_bk = nullptr;
    double *d_pts = nullptr, *d_pts_bk = nullptr;
    EdgeD *d_edges = nullptr;
    orbx_ba_edge *d_raw = nullptr;
    uint8_t *d_active = nullptr, *d_usable = nullptr, *d_front = nullptr;
    double *d_err = nullptr, *d_chi2 = nullptr, *d_rho = nullptr;
    EdgeOut *d_eo = nullptr;
    int32_t *d_coffs = nullptr, *d_clist = nullptr, *d_poffs = nullptr, *d_plist = nullptr, *d_epoint = nullptr,
            *d_cvoffs = nullptr, *d_cvlist = nullptr;
    int2 *d_pairs = nullptr;
    int npairs = 0;
    double *d_Hpp = nullptr, *d_bp = nullptr, *d_Hll = nullptr, *d_bl = nullptr, *d_dinv = nullptr,
           *d_bdinv = nullptr, *d_bdb = nullptr, *d_S = nullptr, *d_bs = nullptr, *d_x = nullptr, *d_db = nullptr;
    int *d_ok = nullptr;
    int32_t *d_efree = nullptr;  // (fast dense mode on a graph without repeated observations) Graph::efree, set_active on the device
    std::vector<int2> pairs_;    // the camera pairs (make_pairs; d_pairs)
    bool pairs_made_ = false;
    void make_pairs();
    int32_t *d_cmap = nullptr;   // free camera x point -> position in its usable list (-1)
    bool use_map = false;        // every (camera, point) observed at most once
    // fast mode's speculative build (lm_optimize): the second linear system
    // (swapped in when the trial is accepted) and the device's acceptance
    EdgeOut *d_eo2 = nullptr;
    double *d_Hpp2 = nullptr, *d_bp2 = nullptr, *d_Hll2 = nullptr, *d_bl2 = nullptr;
    int *d_accept = nullptr;
    void swap_system() {
        std::swap(d_eo, d_eo2); std::swap(d_Hpp, d_Hpp2); std::swap(d_bp, d_bp2);
        std::swap(d_Hll, d_Hll2); std::swap(d_bl, d_bl2);
    }
    hipEvent_t event() {
        if (!ws_.ev && hipEventCreateWithFlags(&ws_.ev, hipEventDisableTiming) != hipSuccess) ws_.ev = nullptr;
        return ws_.ev;
    }
    // fast mode's dense Schur product (k_ba_schur_*): per-point L^-1 and u,
    // the operand M (kp_ x ct_), the chunk partials of the 2x2 tile blocks
    double *d_lu = nullptr, *d_M = nullptr, *d_spart = nullptr;
    int schur_ct_ = 0, schur_ucol_ = 0, schur_kp_ = 0, schur_nch_ = 0, schur_h_ = 0, schur_nblk_ = 0;
    bool dense() const { return fast_ && use_map && dense_schur_on(); }
    std::vector<uint8_t> act_;
    std::vector<int32_t> cv_offs_, cv_list_;   // all edges per free camera (reduce), edge order
    double *d_rho0 = nullptr;                  // rho[0] per edge, contiguous
    int32_t *d_moffs = nullptr, *d_mcnt = nullptr;   // camera pairs' shared-point lists (k_ba_pair_matches)
    int2 *d_mlist = nullptr;
    double *d_terms = nullptr;                 // 36 per shared point of each pair (k_ba_pair_terms)
    double *d_rows = nullptr;                  // records gathered in list order (k_ba_gather_rows), 42 per edge
    int nusable_ = 0;
    int64_t nmatch_ = 0, mbound_ = 0;   // nmatch_: capacity the shared-point kernels are launched over
    uint8_t *hbuf_ = nullptr;                  // pinned readbacks
    double *h_rho0 = nullptr, *h_x = nullptr, *h_bp = nullptr, *h_bl = nullptr, *h_hpp = nullptr, *h_hll = nullptr;
    size_t span_ = 0;      // bytes from d_ok to the end of d_bl
    bool s_zero_ = false;  // d_S's non-pair blocks are zero
    int *h_ok = nullptr;
    // fast mode's device-reduced readback (k_ba_fast_sums): written by the
    // kernel straight into the pinned h_fsum (d_fsum = its device address),
    // visible to the host at the stream synchronisation -- no copy a trial
    double *d_fsum = nullptr, *h_fsum = nullptr;
    double *d_fpart = nullptr;                     // its per-workgroup partials
    double *d_epart = nullptr;                     // k_ba_errors_sums' per-workgroup partials (2 each)
    unsigned *d_fcount = nullptr;                  // its finished-workgroup counter (zeroed by alloc, reset by the last)
    uint8_t *h_stage = nullptr;                // set_active's uploads: flags, then h_coffs_ | clist
    int32_t *h_coffs_ = nullptr;
    size_t schur_bytes() {   // (fast mode) sizes the dense Schur product's buffers
        schur_ct_ = schur_ucol_ = schur_kp_ = schur_nch_ = schur_h_ = schur_nblk_ = 0;
        if (!fast_ || !g_.nf || !dense_schur_on()) return 0;
        const int tce = 2 * ((6 * g_.nf + 31) / 32);   // tile columns of W, even
        schur_h_ = tce / 2;
        schur_ucol_ = 16 * tce;
        schur_ct_ = 16 * (tce + 2);                     // + the u tile and a zero tile (its block's pair)
        schur_nch_ = std::max((3 * g_.npt + kSchurKC - 1) / kSchurKC, 1);
        schur_kp_ = schur_nch_ * kSchurKC;
        schur_nblk_ = schur_h_ * (schur_h_ + 1) / 2 + schur_h_;
        return 8 * (9 * (size_t)std::max(g_.npt, 1) + (size_t)schur_kp_ * schur_ct_ +
                    (size_t)schur_nch_ * schur_nblk_ * 1024) + 256 * 3;
    }
};

// the camera-pair list: free cameras sharing a point (structure of the
// reduced system), from per-camera bitmasks of the cameras it shares a point
// with (nf <= 170: three words); pairs in lexicographic order.  mbound_: the
// shared-point list length with every edge active (a bound for any active
// subset)
void BA::make_pairs() {
    const Graph &g = g_;
    constexpr int kW = 3;
    std::vector<uint64_t> rows((size_t)std::max(g.nf, 1) * kW, 0);
    mbound_ = 0;
    for (int p = 0; p < g.npt; ++p) {
        uint64_t pm[kW] = {0, 0, 0};
        int64_t k = 0;
        for (int t = g.poffs[p]; t < g.poffs[p + 1]; ++t) {
            const int f = g.efree[g.plist[t]];
            if (f >= 0) { pm[f >> 6] |= 1ull << (f & 63); ++k; }
        }
        mbound_ += k * (k + 1) / 2;
        if (!k) continue;
        for (int t = g.poffs[p]; t < g.poffs[p + 1]; ++t) {
            const int f = g.efree[g.plist[t]];
            if (f >= 0)
                for (int w = 0; w < kW; ++w) rows[(size_t)f * kW + w] |= pm[w];
        }
    }
    pairs_.clear();
    for (int a = 0; a < g.nf; ++a)
        for (int b = a; b < g.nf; ++b)
            if (b == a || (rows[(size_t)a * kW + (b >> 6)] >> (b & 63) & 1)) pairs_.push_back(make_int2(a, b));
    npairs = (int)pairs_.size();
    pairs_made_ = true;
}

int BA::alloc() {
    const Graph &g = g_;
    // ORBX_BA_TIMING: the host phases of alloc on stderr (diagnostics)
    static const bool timing = std::getenv("ORBX_BA_TIMING") != nullptr;
    const auto t0 = std::chrono::steady_clock::now();
    auto ms = [&] { return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count(); };
    double t_pairs = 0, t_lists = 0, t_arena = 0;
    const size_t ne = std::max(g.ne, 1), nc = std::max(g.ncam, 1), np = std::max(g.npt, 1), nf = std::max(g.nf, 1);
    // the camera pairs (make_pairs): the fast mode's dense Schur product needs
    // none, so there they are made only if set_active falls back to the merge walk
    const bool lazy_pairs = fast_ && dense_schur_on();
    if (lazy_pairs) {
        pairs_.clear();
        npairs = 0;
        mbound_ = 0;
    } else {
        make_pairs();
    }
    t_pairs = ms();
    // all edges of each free camera in edge order (for Hpp / bp)
    cv_offs_.assign(g.nf + 1, 0);
    for (int e = 0; e < g.ne; ++e) {
        const int f = g.efree[e];
        if (f >= 0) ++cv_offs_[f + 1];
    }
    for (int f = 0; f < g.nf; ++f) cv_offs_[f + 1] += cv_offs_[f];
    cv_list_.assign(std::max(cv_offs_[g.nf], 1), 0);
    {
        std::vector<int> fill(cv_offs_.begin(), cv_offs_.end() - 1);
        for (int e = 0; e < g.ne; ++e) {
            const int f = g.efree[e];
            if (f >= 0) cv_list_[fill[f]++] = e;
        }
    }
    t_lists = ms();
    const size_t n = 6 * nf;
    const size_t pair_cap = lazy_pairs ? nf * (nf + 1) / 2 : (size_t)std::max(npairs, 1);   // (d_pairs)
    const size_t bytes = 256 * 40 + sizeof(Pose) * nc * 2 + 8 * 3 * np * 2 + sizeof(EdgeD) * ne + 3 * ne +
                         8 * ne * 6 + sizeof(EdgeOut) * ne + 4 * (nf + 1 + ne + np + 1 + ne + ne + nf + 1 + ne + ne) + 256 +
                         sizeof(int2) * pair_cap + 8 * (36 * nf + 6 * nf + 9 * np + 3 * np + 9 * np +
                                                                   18 * ne + 6 * ne + n * n + n + n + 3 * np) +
                         4 * nf * np + 8 * ne + 8 * 3 * np + 8 * 42 * ne + sizeof(orbx_ba_edge) * ne + 256 * 6 +
                         schur_bytes() +
                         (fast_ ? sizeof(EdgeOut) * ne + 8 * (36 * nf + 6 * nf + 9 * np + 3 * np) + 256 * 6 +
                                      16 * (std::max(ne, 6 * nf + 3 * np) / kErrSumThreads + 2) + 256 : 0);
    if (ws_.cap < bytes) {
        (void)hipStreamSynchronize(st_);
        if (ws_.dev) (void)hipFree(ws_.dev);
        ws_.dev = nullptr;
        ws_.cap = 0;
        if (hipMalloc(reinterpret_cast<void **>(&ws_.dev), bytes + bytes / 4) != hipSuccess) return ORBX_ENOMEM;
        ws_.cap = bytes + bytes / 4;
    }
    buf_ = ws_.dev;
    uint8_t *p = buf_;
    d_pose = carve<Pose>(p, nc); d_pose_bk = carve<Pose>(p, nc);
    d_pts = carve<double>(p, 3 * np); d_pts_bk = carve<double>(p, 3 * np);
    d_edges = carve<EdgeD>(p, ne);
    d_active = carve<uint8_t>(p, ne); d_usable = carve<uint8_t>(p, ne); d_front = carve<uint8_t>(p, ne);
    d_err = carve<double>(p, 3 * ne); d_chi2 = carve<double>(p, ne); d_rho = carve<double>(p, 2 * ne);
    d_eo = carve<EdgeOut>(p, ne);
    d_coffs = carve<int32_t>(p, nf + 1); d_clist = carve<int32_t>(p, ne);
    d_poffs = carve<int32_t>(p, np + 1); d_plist = carve<int32_t>(p, ne); d_epoint = carve<int32_t>(p, ne);
    d_cvoffs = carve<int32_t>(p, nf + 1); d_cvlist = carve<int32_t>(p, ne);
    d_efree = nullptr;
    if (lazy_pairs) {   // (each free camera observes each point at most once: point lists are by camera)
        bool unique = true;
        for (int q = 0; q < g.npt && unique; ++q) {
            int last = -1;
            for (int t = g.poffs[q]; t < g.poffs[q + 1]; ++t) {
                const int f = g.efree[g.plist[t]];
                if (f >= 0 && f == last) { unique = false; break; }
                if (f >= 0) last = f;
            }
        }
        if (unique) d_efree = carve<int32_t>(p, ne);
    }
    d_pairs = carve<int2>(p, pair_cap);
    d_Hpp = carve<double>(p, 36 * nf);
    d_Hll = carve<double>(p, 9 * np); d_dinv = carve<double>(p, 9 * np);
    d_bdinv = carve<double>(p, 18 * ne); d_bdb = carve<double>(p, 6 * ne);
    d_S = carve<double>(p, n * n); d_bs = carve<double>(p, n);
    // a trial's readback, one span mirrored in the pinned buffer: ok, rho0, x, bp, bl
    d_ok = carve<int>(p, 1);
    d_rho0 = carve<double>(p, ne);
    d_x = carve<double>(p, n + 3 * np);
    d_bp = carve<double>(p, 6 * nf);
    d_bl = carve<double>(p, 3 * np);
    span_ = (size_t)(p - reinterpret_cast<uint8_t *>(d_ok));
    d_cmap = carve<int32_t>(p, nf * np);
    if (schur_ct_) {
        d_lu = carve<double>(p, 9 * np);
        d_M = carve<double>(p, (size_t)schur_kp_ * schur_ct_);
        d_spart = carve<double>(p, (size_t)schur_nch_ * schur_nblk_ * 1024);
    }
    d_fpart = carve<double>(p, 3 * kFastSumBlocks);
    d_fcount = carve<unsigned>(p, 4);
    d_eo2 = nullptr; d_Hpp2 = d_bp2 = d_Hll2 = d_bl2 = nullptr; d_accept = nullptr; d_epart = nullptr;
    if (fast_) {
        d_eo2 = carve<EdgeOut>(p, ne);
        d_Hpp2 = carve<double>(p, 36 * nf); d_bp2 = carve<double>(p, 6 * nf);
        d_Hll2 = carve<double>(p, 9 * np); d_bl2 = carve<double>(p, 3 * np);
        d_accept = carve<int>(p, 1);
        d_epart = carve<double>(p, 2 * (std::max(ne, 6 * nf + 3 * np) / kErrSumThreads + 2));
    }
    d_db = carve<double>(p, 3 * np);
    d_rows = carve<double>(p, 42 * ne);
    d_raw = carve<orbx_ba_edge>(p, ne);
    if ((size_t)(p - buf_) > bytes) return ORBX_ENOMEM;
    {
        const size_t m = n + 3 * np;
        const size_t hb = 8 * (ne + 2 * m + 36 * nf + 9 * np) + 64 + 2 * ne + 4 * (nf + 1 + ne) + 256 * 10;
        if (ws_.hcap < hb) {
            if (ws_.host) (void)hipHostFree(ws_.host);
            ws_.host = nullptr;
            ws_.hcap = 0;
            if (hipHostMalloc(reinterpret_cast<void **>(&ws_.host), hb + hb / 4, hipHostMallocDefault) != hipSuccess)
                return ORBX_ENOMEM;
            ws_.hcap = hb + hb / 4;
        }
        hbuf_ = ws_.host;
        uint8_t *h = hbuf_;
        h_ok = carve<int>(h, 1); h_rho0 = carve<double>(h, ne); h_x = carve<double>(h, m);
        h_bp = carve<double>(h, 6 * nf); h_bl = carve<double>(h, 3 * np);
        h_hpp = carve<double>(h, 36 * nf); h_hll = carve<double>(h, 9 * np);
        h_fsum = carve<double>(h, 12);   // [0, 4): errors / trial sums, [4, 8): read_diag's, [8]: the trial's acceptance
        if (hipHostGetDevicePointer(reinterpret_cast<void **>(&d_fsum), h_fsum, 0) != hipSuccess) return ORBX_EIO;
        h_stage = carve<uint8_t>(h, 2 * ne); h_coffs_ = carve<int32_t>(h, nf + 1 + ne);
        if ((size_t)(h - hbuf_) > hb) return ORBX_ENOMEM;
    }
    // the pairs' shared-point lists (set_active), sized for every edge active
    if (!grow_dev(ws_.moffs, ws_.moffs_cap, 2 * ((size_t)npairs + 1))) return ORBX_ENOMEM;
    d_moffs = ws_.moffs;
    d_mcnt = ws_.moffs + npairs + 1;
    if (mbound_ > ws_.mcap) {
        for (void *x : {(void *)ws_.mlist, (void *)ws_.terms})
            if (x) (void)hipFree(x);
        ws_.mlist = nullptr;
        ws_.terms = nullptr;
        ws_.mcap = 0;
        const size_t m = (size_t)mbound_ * 9 / 8;
        if (hipMalloc(reinterpret_cast<void **>(&ws_.mlist), sizeof(int2) * m) != hipSuccess ||
            hipMalloc(reinterpret_cast<void **>(&ws_.terms), 36 * sizeof(double) * m) != hipSuccess)
            return ORBX_ENOMEM;
        ws_.mcap = (int64_t)m;
    }
    t_arena = ms();
    d_mlist = ws_.mlist;
    d_terms = ws_.terms;
    auto up = [&](void *d, const void *h, size_t b) {
        return b == 0 || hipMemcpyAsync(d, h, b, hipMemcpyHostToDevice, st_) == hipSuccess;
    };
    // the caller's 44-byte edges go up as they are; EdgeD (96 bytes) and the
    // edge -> point list are made on the device
    if (!up(d_raw, g.raw, sizeof(orbx_ba_edge) * g.ne)) return ORBX_EIO;
    if (g.ne)
        hipLaunchKernelGGL(k_ba_edges, dim3((g.ne + 255) / 256), dim3(256), 0, st_, d_raw, g.ne,
                           (double)(float)std::sqrt(5.991), (double)(float)std::sqrt(7.815), d_edges, d_epoint);
    if (hipGetLastError() != hipSuccess || !up(d_poffs, g.poffs.data(), 4 * (g.npt + 1)) ||
        !up(d_plist, g.plist.data(), 4 * g.ne) || !up(d_pairs, pairs_.data(), sizeof(int2) * npairs) ||
        !up(d_cvoffs, cv_offs_.data(), 4 * (g.nf + 1)) || !up(d_cvlist, cv_list_.data(), 4 * cv_list_.size()) ||
        (d_efree && !up(d_efree, g.efree.data(), 4 * (size_t)g.ne)))
        return ORBX_EIO;
    if (timing)
        std::fprintf(stderr, "orbx_local_ba alloc ms: pairs %.3f lists %.3f arena %.3f uploads %.3f\n", t_pairs,
                     t_lists - t_pairs, t_arena - t_lists, ms() - t_arena);
    return ORBX_OK;
}

int BA::upload(const double *pts) {
    if ((fast_ && hipMemsetAsync(d_fcount, 0, 16, st_) != hipSuccess) ||   // (k_ba_fast_sums' counter)
        hipMemcpyAsync(d_pose, g_.poses.data(), sizeof(Pose) * g_.ncam, hipMemcpyHostToDevice, st_) != hipSuccess ||
        (g_.npt && hipMemcpyAsync(d_pts, pts, 24 * (size_t)g_.npt, hipMemcpyHostToDevice, st_) != hipSuccess))
        return ORBX_EIO;
    return ORBX_OK;
}

// active edges; usable = active with a free camera, sorted per camera by
// point.  Host: the flags and per-camera lists, written into pinned staging
// (the caller synchronises the stream before the next set_active); device:
// the point -> list-position map, the pairs' shared-point counts, their scan
// and the lists.  Nothing waits here.
// the second pass's active set from the device's errors: the front flags at
// the current estimate (download's k_ba_errors front_only), the outlier rule,
// then the usable flags and the map (set_active's device path)
int BA::set_active_pass2() {
    const Graph &g = g_;
    s_zero_ = false;
    use_map = true;
    nmatch_ = 0;
    nusable_ = 0;
    if (g.nf && g.npt && hipMemsetAsync(d_cmap, 0xFF, 4 * (size_t)g.nf * g.npt, st_) != hipSuccess) return ORBX_EIO;
    if (!g.ne) return ORBX_OK;
    hipLaunchKernelGGL(k_ba_errors, dim3((g.ne + 63) / 64), dim3(64), 0, st_, d_pose, d_pts, d_edges, g.ne, d_active, 0,
                       1, d_err, d_chi2, d_rho, d_front, nullptr, nullptr);
    hipLaunchKernelGGL(k_ba_pass2_active, dim3((g.ne + 255) / 256), dim3(256), 0, st_, d_edges, g.ne, d_chi2, d_front,
                       d_active);
    hipLaunchKernelGGL(k_ba_usable_map, dim3((g.ne + 255) / 256), dim3(256), 0, st_, d_active, d_efree, d_epoint, g.ne,
                       g.npt, d_usable, d_cmap);
    return hipGetLastError() == hipSuccess ? ORBX_OK : ORBX_EIO;
}

void BA::set_active(const std::vector<uint8_t> &act) {
    static const bool timing = std::getenv("ORBX_BA_TIMING") != nullptr;
    const auto t0 = std::chrono::steady_clock::now();
    act_ = act;
    s_zero_ = false;
    const Graph &g = g_;
    if (d_efree) {   // (fast mode, dense product, no repeated observation: the device builds the set)
        use_map = true;
        nmatch_ = 0;
        nusable_ = 0;
        // (the map is cleared even with no edges: the dense product reads it)
        if (g.nf && g.npt) (void)hipMemsetAsync(d_cmap, 0xFF, 4 * (size_t)g.nf * g.npt, st_);
        if (!g.ne) return;
        std::memcpy(h_stage, act.data(), g.ne);
        (void)hipMemcpyAsync(d_active, h_stage, g.ne, hipMemcpyHostToDevice, st_);
        hipLaunchKernelGGL(k_ba_usable_map, dim3((g.ne + 255) / 256), dim3(256), 0, st_, d_active, d_efree, d_epoint,
                           g.ne, g.npt, d_usable, d_cmap);
        return;
    }
    uint8_t *h_act = h_stage, *h_us = h_stage + g.ne;
    int32_t *h_coffs = h_coffs_, *h_clist = h_coffs_ + g.nf + 1;
    std::fill(h_coffs, h_coffs + g.nf + 1, 0);
    for (int e = 0; e < g.ne; ++e) {
        const int f = g.efree[e];
        h_act[e] = act[e];
        h_us[e] = act[e] && f >= 0;
        if (h_us[e]) ++h_coffs[f + 1];
    }
    for (int f = 0; f < g.nf; ++f) h_coffs[f + 1] += h_coffs[f];
    std::vector<int> fill(h_coffs, h_coffs + std::max(g.nf, 1));
    // point-major walk: each camera's list comes out in ascending point order;
    // a camera seeing a point twice (adjacent: plist is by camera) needs the
    // merge kernel instead of the map
    use_map = true;
    for (int p = 0; p < g.npt; ++p) {
        int last = -1;
        for (int t = g.poffs[p]; t < g.poffs[p + 1]; ++t) {
            const int e = g.plist[t];
            if (!h_us[e]) continue;
            const int f = g.efree[e];
            if (f == last) use_map = false;
            last = f;
            h_clist[fill[f]++] = e;
        }
    }
    nusable_ = h_coffs[g.nf];
    if (timing)
        std::fprintf(stderr, "orbx_local_ba set_active host ms: %.3f\n",
                     std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count());
    (void)hipMemcpyAsync(d_active, h_act, g.ne, hipMemcpyHostToDevice, st_);
    (void)hipMemcpyAsync(d_usable, h_us, g.ne, hipMemcpyHostToDevice, st_);
    (void)hipMemcpyAsync(d_coffs, h_coffs, 4 * (size_t)(g.nf + 1), hipMemcpyHostToDevice, st_);
    if (nusable_) (void)hipMemcpyAsync(d_clist, h_clist, 4 * (size_t)nusable_, hipMemcpyHostToDevice, st_);
    nmatch_ = 0;
    if (!use_map && g.nf && !pairs_made_) {   // (fast mode: the merge walk needs the pairs after all)
        make_pairs();
        if (npairs) (void)hipMemcpyAsync(d_pairs, pairs_.data(), sizeof(int2) * npairs, hipMemcpyHostToDevice, st_);
    }
    if (!use_map || !g.nf) return;
    if (g.npt) {
        (void)hipMemsetAsync(d_cmap, 0xFF, 4 * (size_t)g.nf * g.npt, st_);
        hipLaunchKernelGGL(k_ba_cmap, dim3(g.nf), dim3(256), 0, st_, d_coffs, d_clist, d_epoint, g.npt, d_cmap,
                           fast_ && dense_schur_on() ? 1 : 0);
    }
    if (npairs > 0 && !dense()) {   // the pairs' shared-point lists: count, scan, fill
        hipLaunchKernelGGL(k_ba_pair_matches, dim3((npairs + 3) / 4), dim3(256), 0, st_, d_pairs, npairs, d_coffs,
                           d_clist, d_epoint, d_cmap, g.npt, nullptr, d_mcnt, nullptr);
        hipLaunchKernelGGL(k_ba_scan_counts, dim3(1), dim3(1024), 0, st_, d_mcnt, npairs, d_moffs);
        hipLaunchKernelGGL(k_ba_pair_matches, dim3((npairs + 3) / 4), dim3(256), 0, st_, d_pairs, npairs, d_coffs,
                           d_clist, d_epoint, d_cmap, g.npt, d_moffs, nullptr, d_mlist);
        nmatch_ = mbound_;
    }
}

int BA::errors(bool robust, double *chi_sum) {
    const int ne = g_.ne;
    if (ne) hipLaunchKernelGGL(k_ba_errors, dim3((ne + 63) / 64), dim3(64), 0, st_, d_pose, d_pts, d_edges, ne,
                               d_active, robust ? 1 : 0, 0, d_err, d_chi2, d_rho, d_front, nullptr, nullptr);
    std::vector<double> rho(2 * (size_t)std::max(ne, 1));
    if (hipGetLastError() != hipSuccess ||
        (ne && hipMemcpyAsync(rho.data(), d_rho, 16 * (size_t)ne, hipMemcpyDeviceToHost, st_) != hipSuccess) ||
        hipStreamSynchronize(st_) != hipSuccess)
        return ORBX_EIO;
    double s = 0;   // activeRobustChi2: active edges in order
    for (int e = 0; e < ne; ++e)
        if (act_[e]) s += rho[2 * (size_t)e];
    *chi_sum = s;
    return ORBX_OK;
}

int BA::build(const int *gate) {
    const Graph &g = g_;
    if (g.ne) hipLaunchKernelGGL(k_ba_linearize, dim3((g.ne + 63) / 64), dim3(64), 0, st_, d_pose, d_pts, d_edges,
                                 g.ne, d_active, d_err, d_rho, d_eo, gate);
    if (g.nf) {   // Hpp and bp of each free camera over all its edges, edge order
        constexpr int kEo = sizeof(EdgeOut) / sizeof(double);
        const int nl = cv_offs_[g.nf];
        if (nl)
            hipLaunchKernelGGL((k_ba_gather_rows<42, 1>), dim3((unsigned)(((int64_t)nl * 42 + 255) / 256)), dim3(256), 0,
                               st_, reinterpret_cast<const double *>(d_eo), kEo, d_cvlist, nl, d_active, d_rows, gate);
        if (!sums_ready()) return ORBX_EIO;
        if (fast_)
            hipLaunchKernelGGL((k_ba_stream_sums<42, true>), dim3(g.nf), dim3(kSumThreads), kSumLds, st_, d_rows,
                               d_cvoffs, nullptr, d_Hpp, 36, d_bp, gate);
        else
            hipLaunchKernelGGL((k_ba_stream_sums<42, false>), dim3(g.nf), dim3(kSumThreads), kSumLds, st_, d_rows,
                               d_cvoffs, nullptr, d_Hpp, 36, d_bp, gate);
    }
    if (g.npt) hipLaunchKernelGGL(k_ba_reduce, dim3((g.npt + 3) / 4), dim3(256), 0, st_, d_eo, d_poffs, d_plist,
                                  d_active, g.npt, 1, d_Hll, d_bl, gate);
    return hipGetLastError() == hipSuccess ? ORBX_OK : ORBX_EIO;
}

int BA::solve(double lambda, int *ok) {   // solve_async and its flag, synchronously
    int rc = solve_async(lambda);
    if (rc) return rc;
    int okv = 1;
    if ((g_.nf && hipMemcpyAsync(&okv, d_ok, 4, hipMemcpyDeviceToHost, st_) != hipSuccess) ||
        hipStreamSynchronize(st_) != hipSuccess)
        return ORBX_EIO;
    *ok = okv;
    return ORBX_OK;
}

int BA::errors_async(bool robust, const int *gate) {
    const int ne = g_.ne;
    if (ne) hipLaunchKernelGGL(k_ba_errors, dim3((ne + 63) / 64), dim3(64), 0, st_, d_pose, d_pts, d_edges, ne,
                               d_active, robust ? 1 : 0, 0, d_err, d_chi2, d_rho, d_front, d_rho0, gate);
    return hipGetLastError() == hipSuccess ? ORBX_OK : ORBX_EIO;
}

// The damped system's solve, enqueued: d_ok says whether the Cholesky succeeded
int BA::solve_async(double lambda) {
    const Graph &g = g_;
    const int n = 6 * g.nf;
    if (g.nf && !sums_ready()) return ORBX_EIO;
    // every solve rewrites the pair blocks; the others stay zero unless the
    // in-place factor (n > kCholLds) overwrote them
    if (n && (n > kCholLds || !s_zero_)) {
        if (hipMemsetAsync(d_S, 0, 8 * (size_t)n * n, st_) != hipSuccess) return ORBX_EIO;
        s_zero_ = true;
    }
    if (!g.nf && hipMemsetAsync(d_ok, 0xFF, 4, st_) != hipSuccess) return ORBX_EIO;   // (nothing to factor: ok)
    const bool dn = g.nf && dense();
    if (g.npt) {
        hipLaunchKernelGGL(k_ba_point, dim3((g.npt + 255) / 256), dim3(256), 0, st_, d_Hll, d_bl, g.npt, lambda, d_dinv,
                           d_db, dn ? d_lu : nullptr);
        if (g.ne && !dn)
            hipLaunchKernelGGL(k_ba_point_edges, dim3((g.ne + 63) / 64), dim3(64), 0, st_, d_eo, d_epoint, d_usable,
                               g.ne, d_dinv, d_db, d_bdinv, d_bdb);
    }
    if (dn) {   // S and bs from one dense product (k_ba_schur_*)
        const int64_t tot = (int64_t)schur_kp_ * schur_ct_;
        hipLaunchKernelGGL(k_ba_schur_ops, dim3((unsigned)((tot + 255) / 256)), dim3(256), 0, st_, g.npt, g.nf,
                           schur_ct_, schur_ucol_, schur_kp_, d_cmap, d_eo, g.ne, d_lu, d_M);
        hipLaunchKernelGGL(k_ba_schur_mfma, dim3(schur_nblk_, schur_nch_), dim3(256), 0, st_, d_M, schur_ct_,
                           schur_h_, d_spart);
        hipLaunchKernelGGL(k_ba_schur_sum, dim3((n * n + n + 255) / 256), dim3(256), 0, st_, d_spart, schur_nch_,
                           schur_nblk_, schur_h_, d_Hpp, d_bp, lambda, n, d_S, d_bs);
    } else if (g.nf) {
        if (use_map) {
            const int64_t nterms = 36 * nmatch_;
            if (nterms)
                hipLaunchKernelGGL(k_ba_pair_terms, dim3((unsigned)((nterms + 255) / 256)), dim3(256), 0, st_, d_mlist,
                                   nterms, d_moffs + npairs, d_eo, d_bdinv, d_terms);
            if (fast_)
                hipLaunchKernelGGL(k_ba_pairs_sum<true>, dim3(npairs), dim3(kSumThreads), kSumLds, st_, d_pairs,
                                   d_moffs, d_terms, d_Hpp, lambda, g.nf, d_S);
            else
                hipLaunchKernelGGL(k_ba_pairs_sum<false>, dim3(npairs), dim3(kSumThreads), kSumLds, st_, d_pairs,
                                   d_moffs, d_terms, d_Hpp, lambda, g.nf, d_S);
        }
        else
            hipLaunchKernelGGL(k_ba_pairs, dim3((npairs + 3) / 4), dim3(256), 0, st_, d_pairs, npairs, d_coffs,
                               d_clist, d_epoint, d_eo, d_bdinv, d_Hpp, lambda, g.nf, d_S);
        // bs = bp - sum over the camera's usable edges of B Dinv bl, edge order
        if (nusable_)
            hipLaunchKernelGGL((k_ba_gather_rows<6, 0>), dim3((unsigned)(((int64_t)nusable_ * 6 + 255) / 256)),
                               dim3(256), 0, st_, d_bdb, 6, d_clist, nusable_, nullptr, d_rows, nullptr);
        if (fast_)
            hipLaunchKernelGGL((k_ba_stream_sums<6, true>), dim3(g.nf), dim3(kSumThreads), kSumLds, st_, d_rows,
                               d_coffs, d_bp, d_bs, 6, nullptr, nullptr);
        else
            hipLaunchKernelGGL((k_ba_stream_sums<6, false>), dim3(g.nf), dim3(kSumThreads), kSumLds, st_, d_rows,
                               d_coffs, d_bp, d_bs, 6, nullptr, nullptr);
    }
    if (g.nf) {
        // (fast mode: the augmented-matrix MFMA factorisation, k_ba_chol_fast;
        // the ordered mode keeps the oracle's term order in k_ba_chol_lds.  An
        // unblocked parallel right-looking FMA factorisation, one barrier a
        // column, measured 130 us against the look-ahead kernel's 85 us at 120
        // unknowns: the per-column square root and division on the chain)
        if (fast_ && n <= kCholFastMax && chol_fast_on()) {
            const int R = 16 * ((n + 16) / 16), lb = 8 * (R * (R + 1) + R + 3 * 1024);
            if (lb > 64 * 1024 && hipFuncSetAttribute(reinterpret_cast<const void *>(k_ba_chol_fast),
                                                      hipFuncAttributeMaxDynamicSharedMemorySize, lb) != hipSuccess)
                return ORBX_EIO;
            hipLaunchKernelGGL(k_ba_chol_fast, dim3(1), dim3(512), lb, st_, d_S, n, d_bs, d_x, d_ok, chol_clk());
        } else if (n <= kCholLds) {
            const int lb = 8 * (n * (n + 1) + n);
            if (lb > 64 * 1024 && hipFuncSetAttribute(reinterpret_cast<const void *>(k_ba_chol_lds),
                                                      hipFuncAttributeMaxDynamicSharedMemorySize, lb) != hipSuccess)
                return ORBX_EIO;
            hipLaunchKernelGGL(k_ba_chol_lds, dim3(1), dim3(512), lb, st_, d_S, n, d_bs, d_x, d_ok, chol_clk());
        } else {
            hipLaunchKernelGGL(k_ba_chol, dim3(1), dim3(1024), 0, st_, d_S, n, d_bs, d_x, d_ok);
        }
    }
    if (g.npt && dn) {
        hipLaunchKernelGGL(k_ba_backsub_dense, dim3((g.npt + 3) / 4), dim3(256), 0, st_, d_M, schur_ct_, n, d_x, d_lu,
                           g.npt, d_x + n);
    } else if (g.npt) {
        double *terms = d_rows;   // (free after the reduced right-hand side)
        uint8_t *flag = reinterpret_cast<uint8_t *>(d_rows + 3 * (size_t)std::max(g.ne, 1));
        if (g.ne)
            hipLaunchKernelGGL(k_ba_backsub_terms, dim3((g.ne + 255) / 256), dim3(256), 0, st_, g.ne, d_plist,
                               d_usable, d_eo, d_edges, d_pose, d_x, terms, flag);
        hipLaunchKernelGGL(k_ba_backsub, dim3((g.npt + 63) / 64), dim3(64), 0, st_, d_dinv, d_bl, g.npt, d_poffs,
                           terms, flag, d_x + n);
    }
    return hipGetLastError() == hipSuccess ? ORBX_OK : ORBX_EIO;
}

int BA::update_gated() {   // (the trial's backup of the estimate is written by the update itself)
    const int n = std::max(g_.ncam, g_.npt);
    if (!n) return ORBX_OK;
    hipLaunchKernelGGL(k_ba_update, dim3((n + 255) / 256), dim3(256), 0, st_, d_pose, g_.ncam, d_pts, g_.npt, d_x,
                       d_x + 6 * g_.nf, d_ok, d_pose_bk, d_pts_bk);
    return hipGetLastError() == hipSuccess ? ORBX_OK : ORBX_EIO;
}

// (fast mode: the sums reduced on the device, 32 bytes back instead of the
// per-edge errors and the step; the ordered mode sums on the host in order)
int BA::read_errors() {
    if (fast_) {
        hipLaunchKernelGGL(k_ba_fast_sums, dim3(kFastSumBlocks), dim3(kFastSumThreads), 0, st_, d_rho0, d_active, g_.ne,
                           nullptr, nullptr, nullptr, 0, 0, 0.0, nullptr, nullptr, 0, nullptr, 0, d_fpart, d_fcount, d_fsum,
                           0.0, nullptr);
        return hipGetLastError() == hipSuccess ? ORBX_OK : ORBX_EIO;
    }
    return (g_.ne && hipMemcpyAsync(h_rho0, d_rho0, 8 * (size_t)g_.ne, hipMemcpyDeviceToHost, st_) != hipSuccess)
               ? ORBX_EIO : ORBX_OK;
}

int BA::read_diag() {
    if (fast_) {   // (into slots of its own: read_errors' chi sum in h_fsum[0] stays whatever the order)
        hipLaunchKernelGGL(k_ba_fast_sums, dim3(kFastSumBlocks), dim3(kFastSumThreads), 0, st_, d_rho0, d_active, g_.ne,
                           nullptr, nullptr, nullptr, 0, 0, 0.0, nullptr, d_Hpp, g_.nf, d_Hll, g_.npt, d_fpart, d_fcount,
                           d_fsum + 4, 0.0, nullptr);
        return hipGetLastError() == hipSuccess ? ORBX_OK : ORBX_EIO;
    }
    if ((g_.nf && hipMemcpyAsync(h_hpp, d_Hpp, 8 * 36 * (size_t)g_.nf, hipMemcpyDeviceToHost, st_) != hipSuccess) ||
        (g_.npt && hipMemcpyAsync(h_hll, d_Hll, 8 * 9 * (size_t)g_.npt, hipMemcpyDeviceToHost, st_) != hipSuccess))
        return ORBX_EIO;
    return ORBX_OK;
}

// a trial's readback: the solve flag, the errors at the trial estimate, and
// x and b for computeScale
int BA::errors_trial(bool robust, double lambda, double cur_chi) {
    const int ne = g_.ne, n = 6 * g_.nf, m = n + 3 * g_.npt;
    const int nb = std::max((std::max(ne, m) + kErrSumThreads - 1) / kErrSumThreads, 1);
    hipLaunchKernelGGL(k_ba_errors_sums, dim3(nb), dim3(kErrSumThreads), 0, st_, d_pose, d_pts, d_edges, ne, d_active,
                       robust ? 1 : 0, d_err, d_chi2, d_rho, d_front, d_ok, d_x, d_bp, d_bl, n, m, lambda, d_epart,
                       d_fcount, d_fsum, cur_chi, d_accept);
    return hipGetLastError() == hipSuccess ? ORBX_OK : ORBX_EIO;
}

int BA::read_trial(double lambda, double cur_chi) {
    if (fast_) {
        const int n = 6 * g_.nf, m = n + 3 * g_.npt;
        hipLaunchKernelGGL(k_ba_fast_sums, dim3(kFastSumBlocks), dim3(kFastSumThreads), 0, st_, d_rho0, d_active, g_.ne,
                           d_x, d_bp, d_bl, n, m, lambda, d_ok, nullptr, 0, nullptr, 0, d_fpart, d_fcount, d_fsum,
                           cur_chi, d_accept);
        return hipGetLastError() == hipSuccess ? ORBX_OK : ORBX_EIO;
    }
    return hipMemcpyAsync(h_ok, d_ok, span_, hipMemcpyDeviceToHost, st_) == hipSuccess ? ORBX_OK : ORBX_EIO;
}

double BA::chi_sum_host() const {   // activeRobustChi2: active edges in order
    if (fast_) return h_fsum[0];
    double s = 0;
    for (int e = 0; e < g_.ne; ++e)
        if (act_[e]) s += h_rho0[e];
    return s;
}

double BA::max_diag_host() const {   // computeLambdaInit: max |diagonal| over the free vertices
    if (fast_) return h_fsum[4 + 3];
    double mx = 0.;
    for (int f = 0; f < g_.nf; ++f)
        for (int j = 0; j < 6; ++j) mx = std::max(std::fabs(h_hpp[36 * (size_t)f + 7 * j]), mx);
    for (int p = 0; p < g_.npt; ++p)
        for (int j = 0; j < 3; ++j) mx = std::max(std::fabs(h_hll[9 * (size_t)p + 4 * j]), mx);
    return mx;
}

double BA::scale_host(double lambda) const {   // computeScale: x (lambda x + b), poses then points
    if (fast_) return h_fsum[1];
    const int m = 6 * g_.nf + 3 * g_.npt;
    double s = 0.;
    const int n = 6 * g_.nf;
    for (int j = 0; j < m; ++j) s += h_x[j] * (lambda * h_x[j] + (j < n ? h_bp[j] : h_bl[j - n]));
    return s;
}

int BA::pop() {
    const int n = std::max(g_.ncam, g_.npt);
    if (n) hipLaunchKernelGGL(k_ba_restore, dim3((n + 255) / 256), dim3(256), 0, st_, d_pose, g_.ncam, d_pts, g_.npt,
                              d_pose_bk, d_pts_bk);
    return hipGetLastError() == hipSuccess ? ORBX_OK : ORBX_EIO;
}

// chi2 as last computed (an edge's error is only refreshed while active, and
// a rejected trial's errors stay), the depth test at the current estimate
int BA::download(double *pts, std::vector<double> &chi2, std::vector<uint8_t> &front) {
    if (g_.ne) hipLaunchKernelGGL(k_ba_errors, dim3((g_.ne + 63) / 64), dim3(64), 0, st_, d_pose, d_pts, d_edges,
                                  g_.ne, d_active, 0, 1, d_err, d_chi2, d_rho, d_front, nullptr, nullptr);
    chi2.resize(std::max(g_.ne, 1));
    front.resize(std::max(g_.ne, 1));
    if (hipMemcpyAsync(g_.poses.data(), d_pose, sizeof(Pose) * g_.ncam, hipMemcpyDeviceToHost, st_) != hipSuccess ||
        (g_.npt && hipMemcpyAsync(pts, d_pts, 24 * (size_t)g_.npt, hipMemcpyDeviceToHost, st_) != hipSuccess) ||
        (g_.ne && hipMemcpyAsync(chi2.data(), d_chi2, 8 * (size_t)g_.ne, hipMemcpyDeviceToHost, st_) != hipSuccess) ||
        (g_.ne && hipMemcpyAsync(front.data(), d_front, g_.ne, hipMemcpyDeviceToHost, st_) != hipSuccess) ||
        hipStreamSynchronize(st_) != hipSuccess)
        return ORBX_EIO;
    return ORBX_OK;
}

// OptimizationAlgorithmLevenberg::solve over `iters` iterations
// (optimization_algorithm_levenberg.cpp:60-145); returns iterations run.
// One stream synchronisation per trial: the trial's solve, update and errors
// are enqueued together (update and errors gated on the solve's flag on the
// device) and read back at once.  An iteration that follows an accepted trial
// reuses that trial's errors, which are the errors of the current estimate
// (g2o recomputes them: same values, same sum).
// Fast mode: the device decides each trial's acceptance too (k_ba_fast_sums,
// the host's arithmetic), and the linear system at the trial's estimate is
// built into the second system buffers, gated on that decision, right behind
// the trial: the host waits for the trial's sums alone (an event), and an
// accepted trial's next iteration finds its system built (the buffers swap).
// ORBX_BA_SPEC=0 turns it off.
bool spec_on() {
    static const bool on = env_on("ORBX_BA_SPEC");
    return on;
}
int lm_optimize(BA &ba, int iters, bool robust, int *rc_out) {
    double lambda = 0, ni = 2, currentChi = 0;
    int nBad = 0, it = 0;
    bool fresh = false;   // the device errors are the current estimate's and currentChi their sum
    bool built = false;   // (fast mode) the current estimate's system is built already
    *rc_out = ORBX_OK;
    auto fail = [&](int rc) { *rc_out = rc; return it; };
    const hipEvent_t ev = ba.fast_ && ba.d_eo2 && spec_on() ? ba.event() : nullptr;
    for (; it < iters; ++it) {
        int rc;
        if (!fresh && (rc = ba.errors_async(robust, nullptr))) return fail(rc);
        if (!built && (rc = ba.build())) return fail(rc);
        built = false;
        if (!fresh || it == 0) {
            if ((!fresh && (rc = ba.read_errors())) || (it == 0 && (rc = ba.read_diag()))) return fail(rc);
            if (hipStreamSynchronize(ba.st_) != hipSuccess) return fail(ORBX_EIO);
            if (!fresh) currentChi = ba.chi_sum_host();
            if (it == 0) {
                lambda = 1e-5 * ba.max_diag_host();   // _tau * maxDiagonal
                ni = 2;
                nBad = 0;
            }
        }
        const double iniChi = currentChi;
        double rho = 0;
        int qmax = 0;
        do {
            if ((rc = ba.solve_async(lambda)) || (rc = ba.update_gated()) ||
                (ba.fast_ && ba.d_epart ? (rc = ba.errors_trial(robust, lambda, currentChi))
                                        : ((rc = ba.errors_async(robust, ba.d_ok)) || (rc = ba.read_trial(lambda, currentChi)))))
                return fail(rc);
            if (ev) {
                if (hipEventRecord(ev, ba.st_) != hipSuccess) return fail(ORBX_EIO);
                ba.swap_system();
                rc = ba.build(ba.d_accept);
                ba.swap_system();
                if (rc) return fail(rc);
                if (hipEventSynchronize(ev) != hipSuccess) return fail(ORBX_EIO);
            } else if (hipStreamSynchronize(ba.st_) != hipSuccess) {
                return fail(ORBX_EIO);
            }
            const bool ok = ba.trial_ok();
            // (the reference updates with an unsolved x; the step is rejected either way)
            const double tempChi = ok ? ba.chi_sum_host() : DBL_MAX;
            rho = currentChi - tempChi;
            double sc = ok ? ba.scale_host(lambda) : 0.0;
            sc += 1e-3;
            rho /= sc;
            if (rho > 0 && std::isfinite(tempChi)) {
                double alpha = 1. - std::pow((2 * rho - 1), 3);
                alpha = std::min(alpha, 2. / 3.);
                const double scaleFactor = std::max(1. / 3., alpha);
                lambda *= scaleFactor;
                ni = 2;
                currentChi = tempChi;
                fresh = true;
                if (ev && ba.h_fsum[8] != 0) {   // (the device agreed: its build ran)
                    ba.swap_system();
                    built = true;
                }
            } else {
                lambda *= ni;
                ni *= 2;
                fresh = false;
                if (ok && (rc = ba.pop())) return fail(rc);   // (a failed solve left the estimate alone)
            }
            qmax++;
        } while (rho < 0 && qmax < 10);
        if (qmax == 10 || rho == 0) return it + 1;   // Terminate
        if ((iniChi - currentChi) * 1e3 < iniChi) nBad++;
        else nBad = 0;
        if (nBad >= 3) return it + 1;
    }
    return it;
}

int build_graph(const float *Tcw, const uint8_t *fixed, int ncam, int npt, const orbx_ba_edge *edges, int ne,
                Graph &g) {
    g.ncam = ncam; g.npt = npt; g.ne = ne; g.raw = edges;
    g.poses.resize(ncam);
    int nf = 0;
    for (int c = 0; c < ncam; ++c) {
        pose_from_cv(Tcw + 12 * (size_t)c, g.poses[c]);
        g.poses[c].free_idx = fixed[c] ? -1 : nf++;
        g.poses[c].pad = 0;
    }
    g.nf = nf;
    g.efree.resize(std::max(ne, 1));
    for (int e = 0; e < ne; ++e) {
        if (edges[e].cam < 0 || edges[e].cam >= ncam || edges[e].point < 0 || edges[e].point >= npt) return ORBX_EINVAL;
        g.efree[e] = g.poses[edges[e].cam].free_idx;
    }
    // edges per point, by camera index (stable): bucket by camera, then by point
    std::vector<int> cfill(ncam + 1, 0);
    for (int e = 0; e < ne; ++e) ++cfill[edges[e].cam + 1];
    for (int c = 0; c < ncam; ++c) cfill[c + 1] += cfill[c];
    std::vector<int32_t> bycam(std::max(ne, 1));
    for (int e = 0; e < ne; ++e) bycam[cfill[edges[e].cam]++] = e;
    g.poffs.assign(npt + 1, 0);
    for (int e = 0; e < ne; ++e) ++g.poffs[edges[e].point + 1];
    for (int p = 0; p < npt; ++p) g.poffs[p + 1] += g.poffs[p];
    g.plist.assign(std::max(ne, 1), 0);
    std::vector<int> fill(g.poffs.begin(), g.poffs.end() - 1);
    for (int t = 0; t < ne; ++t) {
        const int e = bycam[t];
        g.plist[fill[edges[e].point]++] = e;
    }
    return ORBX_OK;
}

}  // namespace

extern "C" {

static int local_ba(int device, bool fast, const float *Tcw, const uint8_t *fixed, int ncam, const float *Xw, int npt,
                    const orbx_ba_edge *edges, int ne, int iters1, int iters2, float *Tcw_out, float *Xw_out,
                    uint8_t *outlier, int *iterations) {
    if (ncam < 0 || npt < 0 || ne < 0 || iters1 < 0 || iters2 < 0 || (ncam && (!Tcw || !fixed || !Tcw_out)) ||
        (npt && (!Xw || !Xw_out)) || (ne && (!edges || !outlier)))
        return ORBX_EINVAL;
    // ORBX_BA_TIMING: host-side phase times of this call on stderr (diagnostics)
    static const bool timing = std::getenv("ORBX_BA_TIMING") != nullptr;
    auto now = [] { return std::chrono::steady_clock::now(); };
    auto t_last = now();
    char tbuf[512];
    int tlen = 0;
    auto lap = [&](const char *what) {
        if (!timing) return;
        (void)hipDeviceSynchronize();
        const auto t = now();
        tlen += std::snprintf(tbuf + tlen, sizeof(tbuf) - tlen, " %s %.3f", what,
                              std::chrono::duration<double, std::milli>(t - t_last).count());
        t_last = t;
    };
    Graph g;
    int rc = build_graph(Tcw, fixed, ncam, npt, edges, ne, g);
    if (rc) return rc;
    lap("graph");
    if (g.nf > 170) return ORBX_EINVAL;   // dense reduced system: 6 x 170 rows in one workgroup
    if (hipSetDevice(device) != hipSuccess) return ORBX_ENODEV;
    BAWs &ws = ba_ws(device);
    std::lock_guard<std::mutex> lock(ws.mu);
    if (!ws.st && hipStreamCreateWithFlags(&ws.st, hipStreamNonBlocking) != hipSuccess) return ORBX_EIO;
    const hipStream_t st = ws.st;
    std::vector<double> pts(3 * (size_t)std::max(npt, 1));
    for (size_t i = 0; i < 3 * (size_t)npt; ++i) pts[i] = Xw[i];
    std::vector<uint8_t> out_flags(std::max(ne, 1), 0);
    int its[2] = {0, 0};
    {
        BA ba(g, ws);
        ba.fast_ = fast;
        if ((rc = ba.alloc()) || (rc = ba.upload(pts.data()))) return rc;
        lap("alloc+upload");
        (void)hipMemsetAsync(ba.d_chi2, 0, 8 * (size_t)std::max(ne, 1), st);
        (void)hipMemsetAsync(ba.d_rho, 0, 16 * (size_t)std::max(ne, 1), st);
        (void)hipMemsetAsync(ba.d_err, 0, 24 * (size_t)std::max(ne, 1), st);
        // optimizer.optimize(5) with Huber kernels on every edge (Optimizer.cc:779-781)
        std::vector<uint8_t> act(std::max(ne, 1), 1);
        ba.set_active(act);
        lap("active1");
        its[0] = lm_optimize(ba, iters1, true, &rc);
        lap("lm1");
        std::vector<double> chi2;
        std::vector<uint8_t> front;
        // (fast mode with device-built sets: the second pass's set is made on
        // the device, with no download in between)
        const bool dev2 = !rc && iters2 > 0 && ba.d_efree;
        if (!rc && !dev2) rc = ba.download(pts.data(), chi2, front);
        lap("download1");
        if (!rc && iters2 > 0) {
            // outliers leave the second pass (setLevel(1)); every kernel is dropped (:791-826)
            if (dev2) {
                rc = ba.set_active_pass2();
            } else {
                for (int e = 0; e < ne; ++e) {
                    const double th = g.raw[e].ur >= 0 ? 7.815 : 5.991;
                    if (chi2[e] > th || !front[e]) act[e] = 0;
                }
                ba.set_active(act);
            }
            lap("active2");
            if (!rc) its[1] = lm_optimize(ba, iters2, false, &rc);
            lap("lm2");
            if (!rc) rc = ba.download(pts.data(), chi2, front);
            lap("download2");
        }
        if (!rc)   // the inlier check of :838-870 (an inactive edge keeps its last error)
            for (int e = 0; e < ne; ++e) {
                const double th = g.raw[e].ur >= 0 ? 7.815 : 5.991;
                out_flags[e] = chi2[e] > th || !front[e];
            }
    }
    (void)hipStreamSynchronize(st);
    lap("end");
    if (timing) std::fprintf(stderr, "orbx_local_ba ms:%s\n", tbuf);
    if (rc) return rc;
    for (int c = 0; c < ncam; ++c) pose_to_cv(g.poses[c], Tcw_out + 12 * (size_t)c);
    for (size_t i = 0; i < 3 * (size_t)npt; ++i) Xw_out[i] = (float)pts[i];
    if (ne) std::memcpy(outlier, out_flags.data(), ne);
    if (iterations) { iterations[0] = its[0]; iterations[1] = its[1]; }
    return ORBX_OK;
}

int orbx_local_ba(int device, const float *Tcw, const uint8_t *fixed, int ncam, const float *Xw, int npt,
                  const orbx_ba_edge *edges, int ne, int iters1, int iters2, float *Tcw_out, float *Xw_out,
                  uint8_t *outlier, int *iterations) {
    return local_ba(device, false, Tcw, fixed, ncam, Xw, npt, edges, ne, iters1, iters2, Tcw_out, Xw_out, outlier,
                    iterations);
}

int orbx_local_ba_fast(int device, const float *Tcw, const uint8_t *fixed, int ncam, const float *Xw, int npt,
                       const orbx_ba_edge *edges, int ne, int iters1, int iters2, float *Tcw_out, float *Xw_out,
                       uint8_t *outlier, int *iterations) {
    return local_ba(device, true, Tcw, fixed, ncam, Xw, npt, edges, ne, iters1, iters2, Tcw_out, Xw_out, outlier,
                    iterations);
}

// One linear system of the first pass: computeActiveErrors, buildSystem,
// setLambda(lambda), solve -- the step x (poses, then points) and the robust
// chi2, without the update (test hook for the oracle's identical step).
int orbx_ba_debug_step(int device, const float *Tcw, const uint8_t *fixed, int ncam, const float *Xw, int npt,
                       const orbx_ba_edge *edges, int ne, int robust, double lambda, double *x_out, double *chi2_out,
                       int *solved) {
    if (ncam < 0 || npt < 0 || ne < 0 || !x_out || !chi2_out || !solved || (ncam && (!Tcw || !fixed)) ||
        (npt && !Xw) || (ne && !edges))
        return ORBX_EINVAL;
    Graph g;
    int rc = build_graph(Tcw, fixed, ncam, npt, edges, ne, g);
    if (rc) return rc;
    if (g.nf > 170) return ORBX_EINVAL;
    if (hipSetDevice(device) != hipSuccess) return ORBX_ENODEV;
    BAWs &ws = ba_ws(device);
    std::lock_guard<std::mutex> lock(ws.mu);
    if (!ws.st && hipStreamCreateWithFlags(&ws.st, hipStreamNonBlocking) != hipSuccess) return ORBX_EIO;
    std::vector<double> pts(3 * (size_t)std::max(npt, 1));
    for (size_t i = 0; i < 3 * (size_t)npt; ++i) pts[i] = Xw[i];
    {
        BA ba(g, ws);
        std::vector<uint8_t> act(std::max(ne, 1), 1);
        if (!(rc = ba.alloc()) && !(rc = ba.upload(pts.data()))) {
            ba.set_active(act);
            if (!(rc = ba.errors(robust != 0, chi2_out)) && !(rc = ba.build()) && !(rc = ba.solve(lambda, solved))) {
                const size_t m = 6 * (size_t)g.nf + 3 * (size_t)npt;
                if (m && (hipMemcpy(x_out, ba.d_x, 8 * m, hipMemcpyDeviceToHost) != hipSuccess)) rc = ORBX_EIO;
            }
        }
    }
    return rc;
}

}  // extern "C"
