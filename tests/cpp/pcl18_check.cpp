// Compiled with -Itests/cpp/pcl18 (a PCL-1.8-shaped include tree): the facades must take their
// ICP4R_HAVE_PCL branches and store PCL's own ConstPtr (boost::shared_ptr in PCL 1.8), and the
// ikd facade's point vector must be PCL's aligned-allocator vector.
#include <type_traits>

#include "icp4r/fast_gicp_compat.hpp"
#include "icp4r/ikd_compat.hpp"
#include "icp4r/pcl_compat.hpp"

#ifndef ICP4R_HAVE_PCL
#error "pcl_compat.hpp did not take its ICP4R_HAVE_PCL branch"
#endif
#ifdef ICP4R_STANDALONE
#error "pcl_compat.hpp defined its stand-ins next to PCL's types"
#endif

using Cloud = pcl::PointCloud<pcl::PointXYZI>;
static_assert(std::is_same<pcl::IterativeClosestPoint<pcl::PointXYZI, pcl::PointXYZI>::PointCloudSourceConstPtr,
                           boost::shared_ptr<const Cloud>>::value,
              "ICP facade must store PCL 1.8's boost::shared_ptr<const PointCloud>");
static_assert(std::is_same<fast_gicp::FastGICPSingleThread<pcl::PointXYZI, pcl::PointXYZI>::PointCloudTargetConstPtr,
                           boost::shared_ptr<const Cloud>>::value,
              "GICP facade must store PCL 1.8's boost::shared_ptr<const PointCloud>");
static_assert(std::is_same<KD_TREE<pcl::PointXYZI>::PointVector, Cloud::VectorType>::value,
              "ikd facade's PointVector must be PCL's aligned vector");
static_assert(!std::is_convertible<Cloud::Ptr, std::shared_ptr<const Cloud>>::value,
              "the stand-in Ptr must not be a std::shared_ptr");

int main() {
    Cloud::Ptr src(new Cloud), tgt(new Cloud);
    pcl::IterativeClosestPoint<pcl::PointXYZI, pcl::PointXYZI> icp;
    icp.setInputSource(src);  // Ptr -> ConstPtr, as at iterative_closest_point.cpp:511-512
    icp.setInputTarget(tgt);
    return icp.getInputSource().get() == src.get() ? 0 : 1;
}
