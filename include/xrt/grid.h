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

// SparseGrid: the density in 8^3 leaf bricks, the layout NanoVDB / OpenVDB keep a grid in
// (Src/examples/nanovdb_convert.cpp, Src/grid.h:22-83) — inactive leaves store nothing and
// read as background 0.  Built from bricks directly (e.g. the leaves of a converted .vdb) or
// cut from a dense array (all-zero bricks dropped).  Bounds are the index box of the
// declared dimensions, like DenseGrid, so a SparseGrid cut from a DenseGrid renders
// bit-identically to it (xrt_set_medium_bricks).
class SparseGrid : public DensityGrid {
public:
    static constexpr uint32_t kBrick = 8;
    // table [nbz][nby][nbx] (nb = ceil(n / 8)): brick index or -1; bricks: 512 floats each, [z][y][x]
    SparseGrid(uint32_t nx, uint32_t ny, uint32_t nz, std::vector<int32_t> table, std::vector<float> bricks,
               Vec3f origin = Vec3f(0.0f), float voxelSize = 1.0f);
    static SparseGrid fromDense(uint32_t nx, uint32_t ny, uint32_t nz, const std::vector<float>& data,
                                Vec3f origin = Vec3f(0.0f), float voxelSize = 1.0f);
    AABB getBounds() const override;
    float getMaxDensity() const override;
    uint32_t nx() const { return nx_; }
    uint32_t ny() const { return ny_; }
    uint32_t nz() const { return nz_; }
    uint32_t bricksX() const { return (nx_ + kBrick - 1) / kBrick; }
    uint32_t bricksY() const { return (ny_ + kBrick - 1) / kBrick; }
    uint32_t bricksZ() const { return (nz_ + kBrick - 1) / kBrick; }
    const std::vector<int32_t>& table() const { return table_; }
    const std::vector<float>& bricks() const { return bricks_; }
    uint32_t brickCount() const { return (uint32_t)(bricks_.size() / (kBrick * kBrick * kBrick)); }
    const Vec3f& origin() const { return origin_; }
    float voxelSize() const { return voxel_; }

private:
    uint32_t nx_, ny_, nz_;
    std::vector<int32_t> table_;
    std::vector<float> bricks_;
    Vec3f origin_;
    float voxel_;
};
