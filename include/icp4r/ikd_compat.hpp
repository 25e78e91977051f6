// ikd_compat.hpp — header-only C++ facade: the ikd-Tree map of radar_odometry over icp4r_map.h.
//
// Drop-in for the ikd-Tree calls of /root/reference/src/radar_odometry.cpp (:92, :347-348, :390,
// :396).  A maintainer replaces
//     #include "ikd_Tree.h"
// by
//     #include <icp4r/ikd_compat.hpp>
// and links libicp4r.so; `KD_TREE<pcl::PointXYZI> ikd_Tree(0.3, 0.6, 0.5);` and the Build /
// set_downsample_param / Add_Points / Sector_Search calls stay textually unchanged.
//
// Semantics (include/icp4r/icp4r_map.h): an append-only device store — the node never deletes and
// never adds with downsampling — and Sector_Search as a full filter with the reference's keep test,
// returning the same set as ikd-Tree in insertion order.  Points are repacked to float4
// (x, y, z, intensity) on the way in and restored on the way out, so PCL's 32-byte PointXYZI keeps
// its intensity.  Each KD_TREE owns its own icp4r context (created on first use), so a
// namespace-scope tree, as the node declares it, outlives nothing it depends on.
#pragma once

#include <cstdint>
#include <stdexcept>
#include <string>
#include <vector>

#include "icp4r/icp4r_map.h"
#include "icp4r/pcl_compat.hpp"

namespace icp4r {

template <typename PointType>
class KD_TREE {  // NOLINT — the reference's class name
  public:
    // ikd-Tree's storage type: a std::vector of points (PCL's aligned vector with real PCL/Eigen).
#ifdef ICP4R_HAVE_PCL
    using PointVector = std::vector<PointType, Eigen::aligned_allocator<PointType>>;
#else
    using PointVector = std::vector<PointType>;
#endif

    // delete / balance parameters steer ikd-Tree's rebalancing (no effect on query results);
    // box_length is the downsample box, unused on the node's path (Add_Points(.., false)).
    explicit KD_TREE(float delete_param = 0.5f, float balance_param = 0.6f, float box_length = 0.2f)
        : delete_param_(delete_param), balance_param_(balance_param), downsample_size_(box_length) {}
    KD_TREE(const KD_TREE&) = delete;
    KD_TREE& operator=(const KD_TREE&) = delete;
    ~KD_TREE() {
        if (map_) icp4r_map_destroy(map_);
        if (ctx_) icp4r_destroy(ctx_);
    }

    template <typename Vec>
    void Build(const Vec& point_cloud) {  // NOLINT
        std::vector<float> buf = pack(point_cloud);
        check(icp4r_map_build(map(), buf.data(), (int64_t)point_cloud.size(), 16), "Build");
    }

    void set_downsample_param(float box_length) { downsample_size_ = box_length; }

    template <typename Vec>
    int Add_Points(Vec& PointToAdd, bool downsample_on) {  // NOLINT
        std::vector<float> buf = pack(PointToAdd);
        check(icp4r_map_add_points(map(), buf.data(), (int64_t)PointToAdd.size(), 16, downsample_on ? 1 : 0),
              "Add_Points");
        return 0;  // ikd-Tree returns its downsample counter: 0 without downsampling
    }

    template <typename Vec>
    void Sector_Search(PointType point, const float radius, const float heading, Vec& Storage) {  // NOLINT
        Storage.clear();
        int64_t cap = 0;
        check(icp4r_map_size(map(), &cap), "Sector_Search");
        std::vector<float> out((size_t)(cap > 0 ? cap : 1) * 4);
        const float c[3] = {point.x, point.y, point.z};
        int64_t k = 0;
        check(icp4r_map_sector_search(map(), c, radius, heading, out.data(), cap, &k), "Sector_Search");
        Storage.resize((size_t)k);
        for (int64_t i = 0; i < k; ++i) {
            PointType& p = Storage[(size_t)i];
            p.x = out[4 * i];
            p.y = out[4 * i + 1];
            p.z = out[4 * i + 2];
            p.intensity = out[4 * i + 3];
        }
    }

    int size() {
        int64_t n = 0;
        check(icp4r_map_size(map(), &n), "size");
        return (int)n;
    }

    icp4r_map* handle() { return map(); }

  private:
    icp4r_map* map() {
        if (!map_) {
            check(icp4r_create(&ctx_, 0), "icp4r_create");
            check(icp4r_map_create(ctx_, &map_), "icp4r_map_create");
        }
        return map_;
    }

    template <typename Vec>
    static std::vector<float> pack(const Vec& v) {
        std::vector<float> buf(v.size() * 4 + 4);
        for (size_t i = 0; i < v.size(); ++i) {
            buf[4 * i] = v[i].x;
            buf[4 * i + 1] = v[i].y;
            buf[4 * i + 2] = v[i].z;
            buf[4 * i + 3] = v[i].intensity;
        }
        return buf;
    }

    static void check(int rc, const char* what) {
        if (rc != ICP4R_OK) throw std::runtime_error(std::string("KD_TREE::") + what + ": " + icp4r_last_error());
    }

    float delete_param_, balance_param_, downsample_size_;
    icp4r_ctx* ctx_ = nullptr;
    icp4r_map* map_ = nullptr;
};

}  // namespace icp4r

#ifndef ICP4R_NO_IKD_ALIAS
using icp4r::KD_TREE;
#endif
