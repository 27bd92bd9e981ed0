// tests/cpp/host_geometry_kat.cpp — drives the drop-in host geometry (include/xrt/geometry.h)
// on the inputs of the reference-compiled known answers (tests/golden/ref_kats.json, made by
// oracle/ref_kats.cpp section 10 and the onb section); tests/test_host_geometry.py compares.
//   host_geometry_kat m44   IN OUT : per 4x4 matrix: inverse, m * next matrix, transposed
//   host_geometry_kat frame IN OUT : per (v, t, n, b): worldToLocal, localToWorld
//   host_geometry_kat onb   IN OUT : per vector: normalize, orthonormalBasis t, b
#include <cstdio>
#include <cstring>
#include <vector>

#include "xrt/geometry.h"

static std::vector<float> slurp(const char* path) {
    std::vector<float> v;
    FILE* f = std::fopen(path, "rb");
    if (!f) return v;
    float x;
    while (std::fread(&x, 4, 1, f) == 1) v.push_back(x);
    std::fclose(f);
    return v;
}
static void put3(std::vector<float>& o, const Vec3f& a) { o.push_back(a[0]), o.push_back(a[1]), o.push_back(a[2]); }
static Vec3f get3(const float* p) { return Vec3f(p[0], p[1], p[2]); }

int main(int argc, char** argv) {
    if (argc != 4) return 2;
    const std::vector<float> in = slurp(argv[2]);
    std::vector<float> out;
    if (!std::strcmp(argv[1], "m44")) {
        const size_t n = in.size() / 16;
        std::vector<Matrix44f> ms(n);
        for (size_t q = 0; q < n; ++q)
            for (int i = 0; i < 4; ++i)
                for (int j = 0; j < 4; ++j) ms[q][i][j] = in[16 * q + 4 * i + j];
        for (size_t q = 0; q < n; ++q) {
            const Matrix44f a = ms[q].inverse(), b = ms[q] * ms[(q + 1) % n], c = ms[q].transposed();
            for (const Matrix44f* m : {&a, &b, &c})
                for (int i = 0; i < 4; ++i)
                    for (int j = 0; j < 4; ++j) out.push_back((*m)[i][j]);
        }
    } else if (!std::strcmp(argv[1], "frame")) {
        for (size_t q = 0; q + 12 <= in.size(); q += 12) {
            const Vec3f v = get3(&in[q]), t = get3(&in[q + 3]), n = get3(&in[q + 6]), b = get3(&in[q + 9]);
            put3(out, worldToLocal(v, t, n, b));
            put3(out, localToWorld(v, t, n, b));
        }
    } else if (!std::strcmp(argv[1], "onb")) {
        for (size_t q = 0; q + 3 <= in.size(); q += 3) {
            const Vec3f n = normalize(get3(&in[q]));
            Vec3f t, b;
            orthonormalBasis(n, t, b);
            put3(out, n), put3(out, t), put3(out, b);
        }
    } else {
        return 2;
    }
    FILE* f = std::fopen(argv[3], "wb");
    if (!f) return 1;
    std::fwrite(out.data(), 4, out.size(), f);
    std::fclose(f);
    return 0;
}
