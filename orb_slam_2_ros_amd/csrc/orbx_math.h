// orbx_math.h -- bit-exact device restatements of the float/double library
// routines on the reference path.  Everything is evaluated with explicit
// round-to-nearest intrinsics so no contraction can change a bit.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

namespace orbx {

// cv::fastAtan2 (OpenCV 3.2, core/src/mathfuncs_core.cpp), called at
// ORBextractor.cc:103.  The coefficient products are folded by the compiler in
// IEEE single precision exactly as GCC folds them for the reference build.
constexpr float kRadToDeg = (float)(180 / 3.14159265358979323846);
constexpr float kAtanP1 = 0.9997878412794807f * kRadToDeg;
constexpr float kAtanP3 = -0.3258083974640975f * kRadToDeg;
constexpr float kAtanP5 = 0.1555786518463281f * kRadToDeg;
constexpr float kAtanP7 = -0.04432655554792128f * kRadToDeg;
constexpr float kDblEpsF = (float)2.2204460492503131e-16;  // (float)DBL_EPSILON

__device__ inline float fast_atan2_deg(float y, float x) {
    const float ax = fabsf(x), ay = fabsf(y);
    float a, c, c2;
    if (ax >= ay) {
        c = __fdiv_rn(ay, __fadd_rn(ax, kDblEpsF));
        c2 = __fmul_rn(c, c);
        a = __fmul_rn(__fadd_rn(__fmul_rn(__fadd_rn(__fmul_rn(__fadd_rn(__fmul_rn(kAtanP7, c2), kAtanP5), c2),
                                                     kAtanP3), c2), kAtanP1), c);
    } else {
        c = __fdiv_rn(ax, __fadd_rn(ay, kDblEpsF));
        c2 = __fmul_rn(c, c);
        a = __fsub_rn(90.f,
                      __fmul_rn(__fadd_rn(__fmul_rn(__fadd_rn(__fmul_rn(__fadd_rn(__fmul_rn(kAtanP7, c2), kAtanP5), c2),
                                                              kAtanP3), c2), kAtanP1), c));
    }
    if (x < 0) a = __fsub_rn(180.f, a);
    if (y < 0) a = __fsub_rn(360.f, a);
    return a;
}

// glibc >= 2.27 sincosf (sysdeps/ieee754/flt-32/s_sincosf.c, sincosf.h,
// sincosf_data.c: the ARM optimized-routines algorithm), which the reference's
// cos()/sin() calls resolve to (ORBextractor.cc:113).  Restated for the
// |x| < 120 range (angles here are in [0, 2*pi)); the FMA form equals the
// non-FMA form bit for bit over every float in [0, 6.2832] and equals this
// container's glibc 2.35 sincosf there (exhaustive check).
__device__ inline void glibc_sincosf(float y, float *sinp, float *cosp) {
    // __sincosf_table[0] / [1] differ only in the sign of the cos polynomial
    // (c0..c4); the sign is selected arithmetically (x * +-1 is exact) so no
    // table lives in per-lane scratch.
    constexpr double kHpiInv = 0x1.45F306DC9C883p+23, kHpi = 0x1.921FB54442D18p0;
    constexpr double kC0 = 0x1p0, kC1 = -0x1.ffffffd0c621cp-2, kC2 = 0x1.55553e1068f19p-5,
                     kC3 = -0x1.6c087e89a359dp-10, kC4 = 0x1.99343027bf8c3p-16;
    constexpr double kS1 = -0x1.555545995a603p-3, kS2 = 0x1.1107605230bc4p-7, kS3 = -0x1.994eb3774cf24p-13;
    const uint32_t top = (__float_as_uint(y) >> 20) & 0x7ff;
    double x = y;
    int n = 0;
    double csign = 1.0;
    if (top < 0x3f4u) {            // |y| < pi/4 (top-12-bit compare, as glibc)
        if (top < 0x398u) {        // |y| < 2^-12
            *sinp = y;
            *cosp = 1.0f;
            return;
        }
    } else {
        const double r = __dmul_rn(x, kHpiInv);
        n = ((int32_t)r + 0x800000) >> 24;
        x = __fma_rn(-(double)n, kHpi, x);
        const double sgn = ((n & 3) == 1 || (n & 3) == 2) ? -1.0 : 1.0;   // sign[n & 3]
        if (n & 2) csign = -1.0;                                           // table [1]
        x = __dmul_rn(x, sgn);
    }
    const double c0 = kC0 * csign, c1 = kC1 * csign, c2c = kC2 * csign, c3 = kC3 * csign, c4 = kC4 * csign;
    const double x2 = __dmul_rn(x, x);
    const double x4 = __dmul_rn(x2, x2);
    const double x3 = __dmul_rn(x2, x);
    const double c2 = __fma_rn(x2, c4, c3);
    const double s1 = __fma_rn(x2, kS3, kS2);
    const double c1v = __fma_rn(x2, c1, c0);
    const double x5 = __dmul_rn(x3, x2);
    const double x6 = __dmul_rn(x4, x2);
    const double s = __fma_rn(x3, kS1, x);
    const double c = __fma_rn(x4, c2c, c1v);
    const float sv = (float)__fma_rn(x5, s1, s);
    const float cv = (float)__fma_rn(x6, c2, c);
    if (n & 1) { *sinp = cv; *cosp = sv; }
    else { *sinp = sv; *cosp = cv; }
}

}  // namespace orbx
