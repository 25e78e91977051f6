// radar_odometry's GICP call block (src/radar_odometry.cpp:398-411) compiled against
// include/icp4r/fast_gicp_compat.hpp instead of fast_gicp.  The scan (already associated to the map
// frame) and the submap come from two .bin files in the node's record format; prints what the node
// prints and consumes (converged, score, the final transformation) for tests/test_gicp.py.
#include <cstdio>
#include <fstream>
#include <iostream>

#include "icp4r/fast_gicp_compat.hpp"

static pcl::PointCloud<pcl::PointXYZI>::Ptr read_scan(const char* path) {
    pcl::PointCloud<pcl::PointXYZI>::Ptr c(new pcl::PointCloud<pcl::PointXYZI>);
    std::ifstream f(path, std::ios::binary);
    float rec[5];
    while (f.read(reinterpret_cast<char*>(rec), sizeof(rec))) {
        pcl::PointXYZI p;
        p.x = rec[0];
        p.y = rec[1];
        p.z = rec[2];
        p.intensity = rec[3];
        c->push_back(p);
    }
    return c;
}

int main(int argc, char** argv) {
    if (argc < 3) {
        std::fprintf(stderr, "usage: %s scan_map.bin submap.bin\n", argv[0]);
        return 2;
    }
    pcl::PointCloud<pcl::PointXYZI>::Ptr scan_map = read_scan(argv[1]);
    pcl::PointCloud<pcl::PointXYZI>::Ptr SubMap = read_scan(argv[2]);
    pcl::PointCloud<pcl::PointXYZI>::Ptr Final(new pcl::PointCloud<pcl::PointXYZI>);

    // GICP (radar_odometry.cpp:398-411, verbatim apart from the output lines)
    fast_gicp::FastGICPSingleThread<pcl::PointXYZI, pcl::PointXYZI> fgicp_st;
    fgicp_st.clearTarget();
    fgicp_st.clearSource();
    fgicp_st.setInputTarget(SubMap);
    fgicp_st.setInputSource(scan_map);
    fgicp_st.setCorrespondenceRandomness(5);
    fgicp_st.align(*Final);
    double score = fgicp_st.getFitnessScore();
    Eigen::Matrix<double, 4, 4> icp_result = fgicp_st.getFinalTransformation().cast<double>();

    std::printf("%d %.17g %d %zu\n", (int)fgicp_st.hasConverged(), score, fgicp_st.getNrIterations(), Final->size());
    const Eigen::Matrix<float, 4, 4> T = fgicp_st.getFinalTransformation();
    for (int k = 0; k < 16; ++k) std::printf("%.9g%c", T.data()[k], k == 15 ? '\n' : ' ');
    for (int r = 0; r < 4; ++r)
        for (int c = 0; c < 4; ++c)
            if (icp_result(r, c) != (double)T(r, c)) return 3;
    return 0;
}
