// xrt/grid.h — DensityGrid interface (Src/grid.h:9-15) plus DenseGrid, a dense float grid
// with OpenVDB GridSampler<FloatGrid, BoxSampler>::wsSample semantics (index = (p - origin)
// / voxelSize, voxel centres on integer indices, trilinear, background 0) standing in for
// OpenVDBGrid, whose library and .vdb assets are absent from this image.
#pragma once
#include <vector>

#include "geometry.h"
#include "ray.h"

class DensityGrid {
public:
    virtual ~DensityGrid() = default;
    virtual AABB getBounds() const = 0;
    virtual float getMaxDensity() const = 0;
};

class DenseGrid : public DensityGrid {
public:
    // data laid out [nz][ny][nx]
    DenseGrid(uint32_t nx, uint32_t ny, uint32_t nz, std::vector<float> data, Vec3f origin = Vec3f(0.0f),
              float voxelSize = 1.0f);
    AABB getBounds() const override;     // index bbox of all voxels -> world (voxel centres)
    float getMaxDensity() const override;
    uint32_t nx() const { return nx_; }
    uint32_t ny() const { return ny_; }
    uint32_t nz() const { return nz_; }
    const std::vector<float>& data() const { return data_; }
    const Vec3f& origin() const { return origin_; }
    float voxelSize() const { return voxel_; }

private:
    uint32_t nx_, ny_, nz_;
    std::vector<float> data_;
    Vec3f origin_;
    float voxel_;
};
