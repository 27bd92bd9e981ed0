// xrt/image.h — Image (Src/image.h:8-150): W*H float3, row-major index j + width*i.
// writeMat (OpenCV) is replaced by writePPM/writePFM; gammaCorrection is kept.
#pragma once
#include <cstdint>
#include <string>
#include <vector>

#include "geometry.h"

class Image {
public:
    struct ImageIdx { int i; int j; };
    Image(uint32_t width, uint32_t height) : width(width), height(height), pixels((size_t)width * height) {}
    uint32_t getWidth() const { return width; }
    uint32_t getHeight() const { return height; }
    Vec3f getPixel(uint32_t i, uint32_t j) const { return pixels[j + (size_t)width * i]; }
    void addPixel(uint32_t i, uint32_t j, const Vec3f& rgb) { pixels[j + (size_t)width * i] += rgb; }
    void setPixel(uint32_t i, uint32_t j, const Vec3f& rgb) { pixels[j + (size_t)width * i] = rgb; }
    Image& operator/=(const Vec3f& rgb);
    Image& operator*=(const Vec3f& rgb);
    void gammaCorrection(float gamma);
    bool writePPM(const std::string& filename) const;
    float* data() { return pixels[0].v; }
    const float* data() const { return pixels[0].v; }

private:
    uint32_t width, height;
    std::vector<Vec3f> pixels;
};
static_assert(sizeof(Vec3f) == 12, "Image pixels must be packed float3");
