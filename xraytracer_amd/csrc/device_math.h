// device_math.h — exact-order float math for the gfx950 kernels.
//
// Every helper reproduces the reference's float evaluation as GCC compiles it on x86-64
// (component-wise Vec3 ops, left-to-right sums, no FMA contraction — the whole library is
// built with -ffp-contract=off; fp32 '/' and sqrtf are correctly rounded under hipcc's
// default -fhip-fp32-correctly-rounded-divide-sqrt).  Citations are to /root/reference.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace xrt {

constexpr float kPI = 3.14159265359;             // Src/geometry.h:10 (float)
constexpr float kPI_MUL_2 = 2.0f * kPI;
constexpr float kPI_MUL_4_INV = 1.0f / (4.0f * kPI);
constexpr float kRAY_EPS = 1e-3f;                 // Src/geometry.h:23
constexpr float kEPSILON = 1.19209290e-07f;       // kEpsilon = FLT_EPSILON
constexpr float kINF = 3.40282347e+38f;           // kInfinity = FLT_MAX

struct v3 {
    float x, y, z;
};
__device__ __forceinline__ v3 mk(float x, float y, float z) { return v3{x, y, z}; }
__device__ __forceinline__ v3 xyz(float4 a) { return v3{a.x, a.y, a.z}; }
__device__ __forceinline__ float4 pk(v3 a, float w = 0.0f) { return make_float4(a.x, a.y, a.z, w); }
// Src/geometry.h:174-236
__device__ __forceinline__ v3 operator+(v3 a, v3 b) { return mk(a.x + b.x, a.y + b.y, a.z + b.z); }
__device__ __forceinline__ v3 operator-(v3 a, v3 b) { return mk(a.x - b.x, a.y - b.y, a.z - b.z); }
__device__ __forceinline__ v3 operator*(v3 a, v3 b) { return mk(a.x * b.x, a.y * b.y, a.z * b.z); }
__device__ __forceinline__ v3 operator*(v3 a, float k) { return mk(a.x * k, a.y * k, a.z * k); }
__device__ __forceinline__ v3 operator/(v3 a, float k) { return mk(a.x / k, a.y / k, a.z / k); }
__device__ __forceinline__ v3 operator/(v3 a, v3 b) { return mk(a.x / b.x, a.y / b.y, a.z / b.z); }
__device__ __forceinline__ v3 operator-(v3 a) { return mk(-a.x, -a.y, -a.z); }
// Src/geometry.h:250-261
__device__ __forceinline__ float dot(v3 a, v3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
__device__ __forceinline__ v3 cross(v3 a, v3 b) {
    return mk(a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x);
}
// Src/geometry.cpp:3-16
__device__ __forceinline__ float length(v3 a) { return __builtin_sqrtf(dot(a, a)); }
__device__ __forceinline__ v3 normalize(v3 a) { return a / length(a); }
// std::min / std::max(a, b)
__device__ __forceinline__ float smin(float a, float b) { return (b < a) ? b : a; }
__device__ __forceinline__ float smax(float a, float b) { return (a < b) ? b : a; }
__device__ __forceinline__ float comp(v3 a, uint32_t i) { return i == 0 ? a.x : (i == 1 ? a.y : a.z); }
__device__ __forceinline__ v3 ray_at(v3 o, v3 d, float t) { return o + d * t; }   // Src/ray.h:20

// orthonormalBasis, active branch (Src/geometry.cpp:43-49)
__device__ __forceinline__ void onb(v3 n, v3& t, v3& b) {
    const float sign = __builtin_copysignf(1.0f, n.z);
    const float a = -1.0f / (sign + n.z);
    const float c = n.x * n.y * a;
    t = mk(1.0f + sign * n.x * n.x * a, sign * c, -sign * n.x);
    b = mk(c, sign + n.y * n.y * a, -n.y);
}
// localToWorld (Src/geometry.h:693-701)
__device__ __forceinline__ v3 local_to_world(v3 v, v3 lx, v3 ly, v3 lz) {
    return mk(v.x * lx.x + v.y * ly.x + v.z * lz.x, v.x * lx.y + v.y * ly.y + v.z * lz.y,
              v.x * lx.z + v.y * ly.z + v.z * lz.z);
}

// ---- glibc sinf / cosf ----------------------------------------------------------------
// The reference calls glibc's sinf/cosf (Src/material.h:421-422, light.h:177, medium.h:59).
// glibc 2.35's implementation (sysdeps/ieee754/flt-32/s_sinf.c, s_cosf.c, sincosf.h,
// sincosf_data.c; originally ARM optimized-routines) is not correctly rounded, so a
// device sinf would differ from it in ~1% of cases.  This is a restatement of that
// published algorithm: fast reduction x - n*pi/2 in double for |x| < 120, then a double
// polynomial per quadrant.  The coefficient table below is glibc's __sincosf_table (values
// read from the host libm.so.6 .rodata; layout sign[4], hpi_inv, hpi, c0, c1, s1, c2, s2,
// c3, s3, c4).  tests/test_trig.py checks it bit-for-bit against the host libm over every
// phi = 2*PI*r that the reference's sampler can produce (83,886,080 values) — identical
// for both glibc build variants (with and without FMA contraction).
struct SinCosTab {
    double sign[4], hpi_inv, hpi, c0, c1, s1, c2, s2, c3, s3, c4;
};
static __constant__ const SinCosTab kSinCosTab[2] = {
    {{1.0, -1.0, -1.0, 1.0}, 0x1.45f306dc9c883p+23, 0x1.921fb54442d18p+0, 0x1p0, -0x1.ffffffd0c621cp-2,
     -0x1.555545995a603p-3, 0x1.55553e1068f19p-5, 0x1.1107605230bc4p-7, -0x1.6c087e89a359dp-10,
     -0x1.994eb3774cf24p-13, 0x1.99343027bf8c3p-16},
    {{1.0, -1.0, -1.0, 1.0}, 0x1.45f306dc9c883p+23, 0x1.921fb54442d18p+0, -0x1p0, 0x1.ffffffd0c621cp-2,
     -0x1.555545995a603p-3, -0x1.55553e1068f19p-5, 0x1.1107605230bc4p-7, 0x1.6c087e89a359dp-10,
     -0x1.994eb3774cf24p-13, -0x1.99343027bf8c3p-16}};
__device__ __forceinline__ const SinCosTab& sincos_tab(int i) { return kSinCosTab[i]; }
__device__ __forceinline__ uint32_t abstop12(float x) { return (__float_as_uint(x) >> 20) & 0x7ff; }
__device__ __forceinline__ float sincosf_poly(double x, double x2, const SinCosTab& p, int n) {
    if ((n & 1) == 0) {
        const double x3 = x * x2;
        const double s1 = p.s2 + x2 * p.s3;
        const double x7 = x3 * x2;
        const double s = x + x3 * p.s1;
        return (float)(s + x7 * s1);
    }
    const double x4 = x2 * x2;
    const double c2 = p.c3 + x2 * p.c4;
    const double c1 = p.c0 + x2 * p.c1;
    const double x6 = x4 * x2;
    const double c = c1 + x4 * p.c2;
    return (float)(c + x6 * c2);
}
__device__ __forceinline__ double sincosf_reduce(double x, const SinCosTab& p, int& n) {
    const double r = x * p.hpi_inv;
    n = (((int32_t)r) + 0x800000) >> 24;
    return x - n * p.hpi;
}
__device__ __forceinline__ float glibc_sinf(float y) {
    const float pio4f = 0x1.921FB6p-1f;
    double x = y;
    if (abstop12(y) < abstop12(pio4f)) {
        if (abstop12(y) < abstop12(0x1p-12f)) return y;
        return sincosf_poly(x, x * x, sincos_tab(0), 0);
    }
    if (abstop12(y) < abstop12(120.0f)) {
        int n;
        x = sincosf_reduce(x, sincos_tab(0), n);
        const double s = sincos_tab(0).sign[n & 3];
        return sincosf_poly(x * s, x * x, sincos_tab((n & 2) ? 1 : 0), n);
    }
    return __builtin_sinf(y);  // |x| >= 120: outside every domain this renderer samples
}
__device__ __forceinline__ float glibc_cosf(float y) {
    const float pio4f = 0x1.921FB6p-1f;
    double x = y;
    if (abstop12(y) < abstop12(pio4f)) {
        if (abstop12(y) < abstop12(0x1p-12f)) return 1.0f;
        return sincosf_poly(x, x * x, sincos_tab(0), 1);
    }
    if (abstop12(y) < abstop12(120.0f)) {
        int n;
        x = sincosf_reduce(x, sincos_tab(0), n);
        const double s = sincos_tab(0).sign[n & 3];
        return sincosf_poly(x * s, x * x, sincos_tab((n & 2) ? 1 : 0), n ^ 1);
    }
    return __builtin_cosf(y);
}

}  // namespace xrt
