// Stand-in for <pcl/point_cloud.h> of PCL 1.8 (test fixture, see ../README.md): Ptr / ConstPtr are
// boost::shared_ptr, points is an Eigen::aligned_allocator vector.
#pragma once
#include <Eigen/Core>
#include <boost/shared_ptr.hpp>
#include <cstdint>
#include <vector>

namespace pcl {
template <typename PointT>
class PointCloud {
  public:
    typedef boost::shared_ptr<PointCloud<PointT> > Ptr;
    typedef boost::shared_ptr<const PointCloud<PointT> > ConstPtr;
    typedef std::vector<PointT, Eigen::aligned_allocator<PointT> > VectorType;

    VectorType points;
    uint32_t width = 0, height = 1;
    bool is_dense = true;

    size_t size() const { return points.size(); }
    bool empty() const { return points.empty(); }
    void push_back(const PointT& p) {
        points.push_back(p);
        width = (uint32_t)points.size();
        height = 1;
    }
    void clear() {
        points.clear();
        width = 0;
    }
    void resize(size_t n) {
        points.resize(n);
        width = (uint32_t)n;
        height = 1;
    }
    PointT& operator[](size_t i) { return points[i]; }
    const PointT& operator[](size_t i) const { return points[i]; }
};
}  // namespace pcl
