// Stand-in for <pcl/point_types.h> (test fixture, see ../README.md): PointXYZI in PCL's 32-byte
// layout (PCL_ADD_POINT4D + intensity).
#pragma once

namespace pcl {
struct alignas(16) PointXYZI {
    union {
        float data[4];
        struct {
            float x, y, z;
        };
    };
    union {
        struct {
            float intensity;
        };
        float data_c[4];
    };
    PointXYZI() : data{0.f, 0.f, 0.f, 1.f}, data_c{0.f, 0.f, 0.f, 0.f} {}
};
static_assert(sizeof(PointXYZI) == 32, "PCL PointXYZI is 32 bytes");
}  // namespace pcl
