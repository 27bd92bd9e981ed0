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

// ---- correctly rounded reciprocal / division by a constant, without v_div_* -----------
// IEEE `1.0f / b` compiles to a ~10-instruction div_scale / rcp / 4 fma / div_fmas /
// div_fixup sequence.  For b in the normal range, one Newton step on v_rcp_f32 already
// gives the correctly rounded reciprocal, and Markstein's correction step turns q = x * rc
// (rc = RN(1/c)) into RN(x / c).  Both are checked bit for bit against IEEE division on
// every float input by tests/test_gpu_parity.py (xrt_test_fastdiv); inputs outside the
// checked exponent window take the IEEE division.
template <uint32_t LO, uint32_t HI>
__device__ __forceinline__ bool fd_exp_in(float x) {   // biased exponent in [LO, HI]
    const uint32_t e = (__float_as_uint(x) >> 23) & 0xffu;
    return e - LO <= HI - LO;
}
__device__ __forceinline__ bool fd_normal(float x) { return fd_exp_in<2, 252>(x); }
__device__ __forceinline__ float rcp_newton(float b) {
    const float y0 = __builtin_amdgcn_rcpf(b);
    return __builtin_fmaf(__builtin_fmaf(-b, y0, 1.0f), y0, y0);
}
__device__ __forceinline__ float rcp_rn(float b) {   // == 1.0f / b
    return fd_normal(b) ? rcp_newton(b) : 1.0f / b;
}
__device__ __forceinline__ float div_const_fast(float x, float c, float rc) {
    const float q = x * rc;
    return __builtin_fmaf(__builtin_fmaf(-c, q, x), rc, q);
}
// x / c for a constant c with rc = RN(1/c) (both normal): == x / c.  The residual
// x - c*q is ~2^-24 x, so x's exponent must be >= 25 for it to stay a normal number.
__device__ __forceinline__ float div_const(float x, float c, float rc) {
    return fd_exp_in<25, 248>(x) ? div_const_fast(x, c, rc) : x / c;   // 248: |x / c| < 2^128 for c > 2^-4
}

// orthonormalBasis, active branch (Src/geometry.cpp:43-49)
__device__ __forceinline__ void onb(v3 n, v3& t, v3& b) {
    const float sign = __builtin_copysignf(1.0f, n.z);
    const float a = -rcp_rn(sign + n.z);   // == -1.0f / (sign + n.z)
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
// The two coefficient sets of __sincosf_table differ only in the sign of every cosine
// coefficient (c0..c4), and IEEE negation commutes exactly with * and +, so the second
// set's cosine polynomial is the exact negation of the first's; the quadrant sign table is
// {1, -1, -1, 1}.  Both are applied with selects, so no lane reads a table from memory (a
// per-lane table index made every Lambert sample wait on a global load).
constexpr double kSC_hpi_inv = 0x1.45f306dc9c883p+23, kSC_hpi = 0x1.921fb54442d18p+0;
constexpr double kSC_c0 = 0x1p0, kSC_c1 = -0x1.ffffffd0c621cp-2, kSC_c2 = 0x1.55553e1068f19p-5,
                 kSC_c3 = -0x1.6c087e89a359dp-10, kSC_c4 = 0x1.99343027bf8c3p-16;
constexpr double kSC_s1 = -0x1.555545995a603p-3, kSC_s2 = 0x1.1107605230bc4p-7, kSC_s3 = -0x1.994eb3774cf24p-13;
__device__ __forceinline__ uint32_t abstop12(float x) { return (__float_as_uint(x) >> 20) & 0x7ff; }
// sincosf_poly, sine branch (n even): x + x^3 s1 + x^7 (s2 + x^2 s3)
__device__ __forceinline__ float sincosf_sin_poly(double x, double x2) {
    const double x3 = x * x2;
    const double s1 = kSC_s2 + x2 * kSC_s3;
    const double x7 = x3 * x2;
    const double s = x + x3 * kSC_s1;
    return (float)(s + x7 * s1);
}
// sincosf_poly, cosine branch (n odd) with the first coefficient set
__device__ __forceinline__ double sincosf_cos_poly(double x2) {
    const double x4 = x2 * x2;
    const double c2 = kSC_c3 + x2 * kSC_c4;
    const double c1 = kSC_c0 + x2 * kSC_c1;
    const double x6 = x4 * x2;
    const double c = c1 + x4 * kSC_c2;
    return c + x6 * c2;
}
__device__ __forceinline__ double sincosf_reduce(double x, int& n) {
    const double r = x * kSC_hpi_inv;
    n = (((int32_t)r) + 0x800000) >> 24;
    return x - n * kSC_hpi;
}
// sinf and cosf of one argument together, without divergence.  glibc evaluates, per call,
// sincosf_poly(x * sign[n & 3], x * x, table (n & 2), n) for sinf and the same with n ^ 1
// for cosf, where n even takes the sine polynomial and n odd the cosine one; so for any n
// one of the two results is the sine polynomial and the other the cosine polynomial of the
// same reduced x, and each is evaluated once here, then placed by selects:
//  * the sine polynomial is odd and IEEE negation commutes exactly with * and + (and with
//    the cast to float), so sin_poly(x * sign) == sign * sin_poly(x) bit for bit;
//  * sign[n & 3] = {1, -1, -1, 1}: sinf (n even) takes -sp iff n & 2, cosf (n odd) iff !(n & 2);
//  * both cosine branches negate iff n & 2 (second coefficient set = negated first);
//  * glibc's |y| < pi/4 path skips the reduction: there it yields n == 0 and x - 0 * hpi ==
//    x exactly (|y| * 2/pi * 2^23 < 2^22), so the reduced evaluation is the same numbers;
//  * |y| < 2^-12: sinf returns y, cosf 1.0f.
__device__ __forceinline__ void glibc_sincosf(float y, float& so, float& co) {
    const uint32_t top = abstop12(y);
    if (top >= abstop12(120.0f)) {   // |y| >= 120 or NaN/Inf: outside every sampled domain
        so = __builtin_sinf(y), co = __builtin_cosf(y);
        return;
    }
    int n;
    const double x = sincosf_reduce((double)y, n);
    const double x2 = x * x;
    const float sp = sincosf_sin_poly(x, x2);
    const double cp = sincosf_cos_poly(x2);
    const bool odd = (n & 1) != 0, neg2 = (n & 2) != 0;
    const float cf = (float)(neg2 ? -cp : cp);
    const float s_even = neg2 ? -sp : sp;   // sinf, n even
    const float c_odd = neg2 ? sp : -sp;    // cosf, n odd
    const bool tiny = top < abstop12(0x1p-12f);
    so = tiny ? y : (odd ? cf : s_even);
    co = tiny ? 1.0f : (odd ? c_odd : cf);
}
__device__ __forceinline__ float glibc_sinf(float y) {
    float s, c;
    glibc_sincosf(y, s, c);
    return s;
}
__device__ __forceinline__ float glibc_cosf(float y) {
    float s, c;
    glibc_sincosf(y, s, c);
    return c;
}

// ---- glibc logf / expf ----------------------------------------------------------------
// Used by VolumePathTracing's delta tracking: -std::log(max(1-u, 0)) and
// analyticTransmittance = exp(-sigma*t) (Src/medium.cpp:51, 93-94; geometry.cpp:18-21).
// Restatements of glibc 2.35 e_logf.c / e_expf.c (ARM optimized-routines) as the x86-64
// FMA ifunc variant executes them (the host libm on FMA-capable CPUs); tables are
// __logf_data and __exp2f_data read from the host libm.so.6.  Checked bit-for-bit against
// host libm: logf on every 1-u of a reachable draw u, expf over all negative floats down
// to -104 (tests/test_gpu_parity.py, oracle probe notes in DESIGN.md).
static __constant__ const double kLogfTab[16][2] = {
    {0x1.661ec79f8f3bep+0, -0x1.57bf7808caadep-2}, {0x1.571ed4aaf883dp+0, -0x1.2bef0a7c06ddbp-2},
    {0x1.49539f0f010b0p+0, -0x1.01eae7f513a67p-2}, {0x1.3c995b0b80385p+0, -0x1.b31d8a68224e9p-3},
    {0x1.30d190c8864a5p+0, -0x1.6574f0ac07758p-3}, {0x1.25e227b0b8ea0p+0, -0x1.1aa2bc79c8100p-3},
    {0x1.1bb4a4a1a343fp+0, -0x1.a4e76ce8c0e5ep-4}, {0x1.12358f08ae5bap+0, -0x1.1973c5a611cccp-4},
    {0x1.0953f419900a7p+0, -0x1.252f438e10c1ep-5}, {0x1.0000000000000p+0, 0x0.0p+0},
    {0x1.e608cfd9a47acp-1, 0x1.aa5aa5df25984p-5}, {0x1.ca4b31f026aa0p-1, 0x1.c5e53aa362eb4p-4},
    {0x1.b2036576afce6p-1, 0x1.526e57720db08p-3}, {0x1.9c2d163a1aa2dp-1, 0x1.bc2860d224770p-3},
    {0x1.886e6037841edp-1, 0x1.1058bc8a07ee1p-2}, {0x1.767dcf5534862p-1, 0x1.4043057b6ee09p-2}};
__device__ __forceinline__ float glibc_logf(float x) {
    const double Ln2 = 0x1.62e42fefa39efp-1, A0 = -0x1.00ea348b88334p-2, A1 = 0x1.5575b0be00b6ap-2,
                 A2 = -0x1.ffffef20a4123p-2;
    uint32_t ix = __float_as_uint(x);
    if (ix == 0x3f800000u) return 0.0f;
    if (ix - 0x00800000u >= 0x7f800000u - 0x00800000u) {
        if (ix * 2 == 0) return -__builtin_inff();
        if (ix == 0x7f800000u) return x;
        if ((ix & 0x80000000u) || ix * 2 >= 0xff000000u) return __builtin_nanf("");
        ix = __float_as_uint(x * 0x1p23f);
        ix -= 23u << 23;
    }
    const uint32_t tmp = ix - 0x3f330000u;
    const int i = (tmp >> (23 - 4)) % 16;
    const int k = (int32_t)tmp >> 23;
    const uint32_t iz = ix - (tmp & 0xff800000u);
    const double invc = kLogfTab[i][0], logc = kLogfTab[i][1];
    const double z = (double)__uint_as_float(iz);
    const double r = __builtin_fma(z, invc, -1.0);
    const double y0 = __builtin_fma((double)k, Ln2, logc);
    const double r2 = r * r;
    double y = __builtin_fma(A1, r, A2);
    y = __builtin_fma(A0, r2, y);
    y = __builtin_fma(y, r2, y0 + r);
    return (float)y;
}
static __constant__ const uint64_t kExp2fTab[32] = {
    0x3ff0000000000000, 0x3fefd9b0d3158574, 0x3fefb5586cf9890f, 0x3fef9301d0125b51, 0x3fef72b83c7d517b,
    0x3fef54873168b9aa, 0x3fef387a6e756238, 0x3fef1e9df51fdee1, 0x3fef06fe0a31b715, 0x3feef1a7373aa9cb,
    0x3feedea64c123422, 0x3feece086061892d, 0x3feebfdad5362a27, 0x3feeb42b569d4f82, 0x3feeab07dd485429,
    0x3feea47eb03a5585, 0x3feea09e667f3bcd, 0x3fee9f75e8ec5f74, 0x3feea11473eb0187, 0x3feea589994cce13,
    0x3feeace5422aa0db, 0x3feeb737b0cdc5e5, 0x3feec49182a3f090, 0x3feed503b23e255d, 0x3feee89f995ad3ad,
    0x3feeff76f2fb5e47, 0x3fef199bdd85529c, 0x3fef3720dcef9069, 0x3fef5818dcfba487, 0x3fef7c97337b9b5f,
    0x3fefa4afa2a490da, 0x3fefd0765b6e4540};
__device__ __forceinline__ float glibc_expf(float x) {
    const double SHIFT = 0x1.8p+52, InvLn2N = 0x1.71547652b82fep+5, C0 = 0x1.c6af84b912394p-20,
                 C1 = 0x1.ebfce50fac4f3p-13, C2 = 0x1.62e42ff0c52d6p-6;
    const double xd = (double)x;
    const uint32_t top = __float_as_uint(x) >> 20;
    const uint32_t abstop = top & 0x7ff;
    if (abstop >= (__float_as_uint(88.0f) >> 20)) {
        if (__float_as_uint(x) == 0xff800000u) return 0.0f;
        if (abstop >= (0x7f800000u >> 20)) return x + x;
        if (x > 0x1.62e42ep6f) return __builtin_inff();
        if (x < -0x1.9fe368p6f) return 0.0f;
    }
    double kd = __builtin_fma(InvLn2N, xd, SHIFT);
    const uint64_t ki = (uint64_t)__double_as_longlong(kd);
    kd -= SHIFT;
    const double r = __builtin_fma(InvLn2N, xd, -kd);
    uint64_t t = kExp2fTab[ki % 32];
    t += ki << (52 - 5);
    const double s = __longlong_as_double((long long)t);
    const double zz = __builtin_fma(C0, r, C1);
    const double r2 = r * r;
    double y = __builtin_fma(C2, r, 1.0);
    y = __builtin_fma(zz, r2, y);
    return (float)(y * s);
}

// ---- glibc powf -----------------------------------------------------------------------
// Image::gammaCorrection's std::pow(float, float) (Src/image.h:80-90).  Restatement of
// glibc 2.35 e_powf.c (ARM optimized-routines) as the x86-64 FMA ifunc variant executes it:
// log2 of x in double from __powf_log2_data (16-entry table + order-5 polynomial, the
// table identical to __log2f_data's), y * log2(x), then exp2 from __exp2f_data (tab,
// shift_scaled, unscaled poly); tables read from the host libm.so.6.  Special cases
// (zero / inf / nan, negative x with integer y, subnormal x) follow the published code.
// Checked bit-for-bit against host powf (tests/test_gpu_parity.py, xrt_test_powf).
static __constant__ const double kPowfLog2Tab[16][2] = {
    {0x1.661ec79f8f3bep+0, -0x1.efec65b963019p-2}, {0x1.571ed4aaf883dp+0, -0x1.b0b6832d4fca4p-2},
    {0x1.49539f0f010b0p+0, -0x1.7418b0a1fb77bp-2}, {0x1.3c995b0b80385p+0, -0x1.39de91a6dcf7bp-2},
    {0x1.30d190c8864a5p+0, -0x1.01d9bf3f2b631p-2}, {0x1.25e227b0b8ea0p+0, -0x1.97c1d1b3b7af0p-3},
    {0x1.1bb4a4a1a343fp+0, -0x1.2f9e393af3c9fp-3}, {0x1.12358f08ae5bap+0, -0x1.960cbbf788d5cp-4},
    {0x1.0953f419900a7p+0, -0x1.a6f9db6475fcep-5}, {0x1.0000000000000p+0, 0x0.0p+0},
    {0x1.e608cfd9a47acp-1, 0x1.338ca9f24f53dp-4}, {0x1.ca4b31f026aa0p-1, 0x1.476a9543891bap-3},
    {0x1.b2036576afce6p-1, 0x1.e840b4ac4e4d2p-3}, {0x1.9c2d163a1aa2dp-1, 0x1.40645f0c6651cp-2},
    {0x1.886e6037841edp-1, 0x1.88e9c2c1b9ff8p-2}, {0x1.767dcf5534862p-1, 0x1.ce0a44eb17bccp-2}};
__device__ __forceinline__ bool powf_zeroinfnan(uint32_t i) { return 2u * i - 1u >= 2u * 0x7f800000u - 1u; }
// 0: not an integer, 1: odd integer, 2: even integer (checkint)
__device__ __forceinline__ int powf_checkint(uint32_t iy) {
    const int e = (int)(iy >> 23 & 0xff);
    if (e < 0x7f) return 0;
    if (e > 0x7f + 23) return 2;
    if (iy & ((1u << (0x7f + 23 - e)) - 1u)) return 0;
    if (iy & (1u << (0x7f + 23 - e))) return 1;
    return 2;
}
__device__ __forceinline__ float glibc_powf(float x, float y) {
    const double A0 = 0x1.27616c9496e0bp-2, A1 = -0x1.71969a075c67ap-2, A2 = 0x1.ec70a6ca7baddp-2,
                 A3 = -0x1.7154748bef6c8p-1, A4 = 0x1.71547652ab82bp+0;
    const double SHIFT = 0x1.8p+47, C0 = 0x1.c6af84b912394p-5, C1 = 0x1.ebfce50fac4f3p-3,
                 C2 = 0x1.62e42ff0c52d6p-1;
    uint32_t sign_bias = 0;
    uint32_t ix = __float_as_uint(x);
    const uint32_t iy = __float_as_uint(y);
    if (ix - 0x00800000u >= 0x7f800000u - 0x00800000u || powf_zeroinfnan(iy)) {
        if (powf_zeroinfnan(iy)) {
            if (2u * iy == 0u) return 1.0f;   // signalling-NaN x aside
            if (ix == 0x3f800000u) return 1.0f;
            if (2u * ix > 2u * 0x7f800000u || 2u * iy > 2u * 0x7f800000u) return x + y;
            if (2u * ix == 2u * 0x3f800000u) return 1.0f;
            if ((2u * ix < 2u * 0x3f800000u) == !(iy & 0x80000000u)) return 0.0f;
            return y * y;
        }
        if (powf_zeroinfnan(ix)) {
            float x2 = x * x;
            if ((ix & 0x80000000u) && powf_checkint(iy) == 1) x2 = -x2;
            return (iy & 0x80000000u) ? 1.0f / x2 : x2;
        }
        if (ix & 0x80000000u) {   // finite x < 0
            const int yint = powf_checkint(iy);
            if (yint == 0) return __builtin_nanf("");
            if (yint == 1) sign_bias = 1u << (5 + 11);
            ix &= 0x7fffffffu;
        }
        if (ix < 0x00800000u) {   // subnormal x
            ix = __float_as_uint(__uint_as_float(ix) * 0x1p23f);
            ix &= 0x7fffffffu;
            ix -= 23u << 23;
        }
    }
    // log2_inline
    const uint32_t tmp = ix - 0x3f330000u;
    const int i = (int)((tmp >> (23 - 4)) % 16);
    const uint32_t top = tmp & 0xff800000u;
    const uint32_t iz = ix - top;
    const int k = (int32_t)top >> 23;
    const double invc = kPowfLog2Tab[i][0], logc = kPowfLog2Tab[i][1];
    const double z = (double)__uint_as_float(iz);
    const double r = __builtin_fma(z, invc, -1.0);
    const double y0 = logc + (double)k;
    const double r2 = r * r;
    double yy = __builtin_fma(A0, r, A1);
    const double p = __builtin_fma(A2, r, A3);
    const double r4 = r2 * r2;
    double q = __builtin_fma(A4, r, y0);
    q = __builtin_fma(p, r2, q);
    yy = __builtin_fma(yy, r4, q);
    const double ylogx = (double)y * yy;
    if (((uint64_t)__double_as_longlong(ylogx) >> 47 & 0xffff) >= ((uint64_t)__double_as_longlong(126.0) >> 47)) {
        if (ylogx > 0x1.fffffffd1d571p+6) return sign_bias ? -__builtin_inff() : __builtin_inff();
        if (ylogx <= -150.0) return sign_bias ? -0.0f : 0.0f;
    }
    // exp2_inline
    double kd = ylogx + SHIFT;
    const uint64_t ki = (uint64_t)__double_as_longlong(kd);
    kd -= SHIFT;
    const double rr = ylogx - kd;
    uint64_t t = kExp2fTab[ki % 32];
    const uint64_t ski = ki + sign_bias;
    t += ski << (52 - 5);
    const double s = __longlong_as_double((long long)t);
    const double zz = __builtin_fma(C0, rr, C1);
    const double rr2 = rr * rr;
    double e = __builtin_fma(C2, rr, 1.0);
    e = __builtin_fma(zz, rr2, e);
    return (float)(e * s);
}

}  // namespace xrt
