// xrt/geometry.h — value types of the reference API (Src/geometry.h): Vec2/Vec3/Matrix44
// with the same names, constructors and operator semantics (component-wise float ops,
// row-vector matrices), so scene-building code written against the reference compiles
// unchanged.  Only what scene construction needs is provided; the ray-tracing math
// itself runs on the GPU (xraytracer_amd/csrc/device_math.h).
#pragma once

#include <cmath>
#include <cstdint>
#include <utility>

constexpr float PI = 3.14159265359;                  // Src/geometry.h:10
constexpr float PI_MUL_2 = 2.0f * PI;
constexpr float PI_INV = 1.0f / PI;
constexpr float RAY_EPS = 1e-3f;                     // Src/geometry.h:23

inline float deg2rad(float deg) { return deg / 180.0f * PI; }   // Src/geometry.h:26
inline float rad2deg(float rad) { return 180.0f * rad / PI; }

template <typename T>
struct Vec2 {
    T v[2];
    Vec2() : v{0, 0} {}
    Vec2(T a) : v{a, a} {}
    Vec2(T a, T b) : v{a, b} {}
    T operator[](int i) const { return v[i]; }
    T& operator[](int i) { return v[i]; }
};

template <typename T>
struct Vec3 {
    T v[3];
    static constexpr int dim = 3;
    Vec3() : v{0, 0, 0} {}
    Vec3(T a) : v{a, a, a} {}
    Vec3(T a, T b, T c) : v{a, b, c} {}
    T operator[](int i) const { return v[i]; }
    T& operator[](int i) { return v[i]; }
    const T* getPtr() const { return v; }
    Vec3 operator-() const { return Vec3(-v[0], -v[1], -v[2]); }
    Vec3& operator+=(const Vec3& o) { for (int i = 0; i < 3; ++i) v[i] += o.v[i]; return *this; }
    Vec3& operator*=(const Vec3& o) { for (int i = 0; i < 3; ++i) v[i] *= o.v[i]; return *this; }
    Vec3& operator/=(const Vec3& o) { for (int i = 0; i < 3; ++i) v[i] /= o.v[i]; return *this; }
};

#define XRT_VEC3_BINOP(OP)                                                                         \
    template <typename T>                                                                          \
    inline Vec3<T> operator OP(const Vec3<T>& a, const Vec3<T>& b) {                               \
        return Vec3<T>(a[0] OP b[0], a[1] OP b[1], a[2] OP b[2]);                                  \
    }                                                                                              \
    template <typename T>                                                                          \
    inline Vec3<T> operator OP(const Vec3<T>& a, float k) {                                        \
        return Vec3<T>(a[0] OP k, a[1] OP k, a[2] OP k);                                           \
    }
XRT_VEC3_BINOP(+)
XRT_VEC3_BINOP(-)
XRT_VEC3_BINOP(*)
XRT_VEC3_BINOP(/)
#undef XRT_VEC3_BINOP
template <typename T>
inline Vec3<T> operator*(float k, const Vec3<T>& a) { return a * k; }
template <typename T>
inline Vec3<T> operator+(float k, const Vec3<T>& a) { return a + k; }
template <typename T>
inline Vec3<T> operator/(float k, const Vec3<T>& a) { return Vec3<T>(k / a[0], k / a[1], k / a[2]); }

template <typename T>
inline T dot(const Vec3<T>& a, const Vec3<T>& b) { return a[0] * b[0] + a[1] * b[1] + a[2] * b[2]; }
template <typename T>
inline Vec3<T> cross(const Vec3<T>& a, const Vec3<T>& b) {
    return Vec3<T>(a[1] * b[2] - a[2] * b[1], a[2] * b[0] - a[0] * b[2], a[0] * b[1] - a[1] * b[0]);
}

using Vec2f = Vec2<float>;
using Vec3f = Vec3<float>;
using Vec3ui = Vec3<uint32_t>;

inline float length2(const Vec3f& a) { return dot(a, a); }
inline float length(const Vec3f& a) { return std::sqrt(dot(a, a)); }
inline Vec3f normalize(const Vec3f& a) { return a / length(a); }   // 3 divides, Src/geometry.cpp:13-16

// Row-vector 4x4 matrix (Src/geometry.h:280-631): points transform as p * M.
template <typename T>
class Matrix44 {
public:
    T x[4][4] = {{1, 0, 0, 0}, {0, 1, 0, 0}, {0, 0, 1, 0}, {0, 0, 0, 1}};
    Matrix44() {}
    Matrix44(T a, T b, T c, T d, T e, T f, T g, T h, T i, T j, T k, T l, T m, T n, T o, T p)
        : x{{a, b, c, d}, {e, f, g, h}, {i, j, k, l}, {m, n, o, p}} {}
    const T* operator[](uint8_t r) const { return x[r]; }
    T* operator[](uint8_t r) { return x[r]; }
    // point transform with homogeneous divide (Src/geometry.h:465-478)
    template <typename S>
    void multVecMatrix(const Vec3<S>& s, Vec3<S>& d) const {
        S a = s[0] * x[0][0] + s[1] * x[1][0] + s[2] * x[2][0] + x[3][0];
        S b = s[0] * x[0][1] + s[1] * x[1][1] + s[2] * x[2][1] + x[3][1];
        S c = s[0] * x[0][2] + s[1] * x[1][2] + s[2] * x[2][2] + x[3][2];
        S w = s[0] * x[0][3] + s[1] * x[1][3] + s[2] * x[2][3] + x[3][3];
        d = Vec3<S>(a / w, b / w, c / w);
    }
    // direction transform (Src/geometry.h:486-498)
    template <typename S>
    void multDirMatrix(const Vec3<S>& s, Vec3<S>& d) const {
        d = Vec3<S>(s[0] * x[0][0] + s[1] * x[1][0] + s[2] * x[2][0],
                    s[0] * x[0][1] + s[1] * x[1][1] + s[2] * x[2][1],
                    s[0] * x[0][2] + s[1] * x[1][2] + s[2] * x[2][2]);
    }
    // c = a * b, every entry summed left to right over k (Src/geometry.h:314-385)
    static void multiply(const Matrix44& a, const Matrix44& b, Matrix44& c) {
        for (int i = 0; i < 4; ++i)
            for (int j = 0; j < 4; ++j)
                c.x[i][j] = a.x[i][0] * b.x[0][j] + a.x[i][1] * b.x[1][j] + a.x[i][2] * b.x[2][j] + a.x[i][3] * b.x[3][j];
    }
    Matrix44 operator*(const Matrix44& b) const {
        Matrix44 c;
        multiply(*this, b, c);
        return c;
    }
    Matrix44 transposed() const {   // Src/geometry.h:397-425
        Matrix44 t;
        for (int i = 0; i < 4; ++i)
            for (int j = 0; j < 4; ++j) t.x[i][j] = x[j][i];
        return t;
    }
    Matrix44& transpose() { return *this = transposed(); }
    // Gauss-Jordan inverse (Src/geometry.h:509-590): partial pivoting on |t[j][i]| over
    // columns 0..2 (a strictly larger magnitude moves the pivot), row reduction with
    // f = t[j][i] / t[i][i], then backward substitution dividing each row by its diagonal.
    // A zero pivot returns the identity, as the reference does.
    Matrix44 inverse() const {
        Matrix44 s, t(*this);
        for (int i = 0; i < 3; ++i) {
            int piv = i;
            T best = t.x[i][i] < 0 ? -t.x[i][i] : t.x[i][i];
            for (int j = i + 1; j < 4; ++j) {
                const T a = t.x[j][i] < 0 ? -t.x[j][i] : t.x[j][i];
                if (a > best) piv = j, best = a;
            }
            if (best == 0) return Matrix44();
            if (piv != i)
                for (int j = 0; j < 4; ++j) {
                    std::swap(t.x[i][j], t.x[piv][j]);
                    std::swap(s.x[i][j], s.x[piv][j]);
                }
            for (int j = i + 1; j < 4; ++j) {
                const T f = t.x[j][i] / t.x[i][i];
                for (int k = 0; k < 4; ++k) {
                    t.x[j][k] -= f * t.x[i][k];
                    s.x[j][k] -= f * s.x[i][k];
                }
            }
        }
        for (int i = 3; i >= 0; --i) {
            T f = t.x[i][i];
            if (f == 0) return Matrix44();
            for (int j = 0; j < 4; ++j) {
                t.x[i][j] /= f;
                s.x[i][j] /= f;
            }
            for (int j = 0; j < i; ++j) {
                f = t.x[j][i];
                for (int k = 0; k < 4; ++k) {
                    t.x[j][k] -= f * t.x[i][k];
                    s.x[j][k] -= f * s.x[i][k];
                }
            }
        }
        return s;
    }
    const Matrix44& invert() { return *this = inverse(); }
};
using Matrix44f = Matrix44<float>;

template <typename S>
inline Vec3<S> multVecMatrix(const Vec3<S>& s, const Matrix44<S>& m) { Vec3<S> d; m.multVecMatrix(s, d); return d; }
template <typename S>
inline Vec3<S> multDirMatrix(const Vec3<S>& s, const Matrix44<S>& m) { Vec3<S> d; m.multDirMatrix(s, d); return d; }

// Src/geometry.cpp:23-49 (the active #else branch; Duff et al.'s branchless basis): t and b
// complete n to an orthonormal frame; n[2] == -0 takes sign -1, as copysign does.
inline void orthonormalBasis(const Vec3f& n, Vec3f& t, Vec3f& b) {
    const float sign = std::copysign(1.0f, n[2]);
    const float a = -1.0f / (sign + n[2]);
    const float c = n[0] * n[1] * a;
    t = Vec3f(1.0f + sign * n[0] * n[0] * a, sign * c, -sign * n[0]);
    b = Vec3f(c, sign + n[1] * n[1] * a, -n[1]);
}

// direction into / out of the frame (lx, ly, lz) (Src/geometry.h:686-701)
inline Vec3f worldToLocal(const Vec3f& v, const Vec3f& lx, const Vec3f& ly, const Vec3f& lz) {
    return Vec3f(dot(v, lx), dot(v, ly), dot(v, lz));
}
inline Vec3f localToWorld(const Vec3f& v, const Vec3f& lx, const Vec3f& ly, const Vec3f& lz) {
    return Vec3f(v[0] * lx[0] + v[1] * ly[0] + v[2] * lz[0], v[0] * lx[1] + v[1] * ly[1] + v[2] * lz[1],
                 v[0] * lx[2] + v[1] * ly[2] + v[2] * lz[2]);
}

// componentwise exp (Src/geometry.cpp:18-21)
inline Vec3f exp(const Vec3f& v) { return Vec3f(std::exp(v[0]), std::exp(v[1]), std::exp(v[2])); }

enum class MaterialType { Lambert, Metals, Glass, Luminous, Unknow };   // Src/geometry.h:703
