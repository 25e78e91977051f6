// The reference node's ICP call sequence (src/iterative_closest_point.cpp:510-521), compiled against
// include/icp4r/pcl_compat.hpp instead of <pcl/registration/icp.h>.  Clouds are built the way the
// node builds them (:64-82 reader, :354-385 parse, :404-406 push of every point), from two scans in
// the reference's .bin format.  Prints the outputs for tests/test_gpu_parity.py to compare.
#include <cstdio>
#include <fstream>
#include <iostream>
#include <vector>

#include "icp4r/pcl_compat.hpp"

static std::vector<float> read_radar_data(const char* path) {
    std::ifstream f(path, std::ifstream::in | std::ifstream::binary);
    if (!f) return {};
    f.seekg(0, std::ios::end);
    const size_t num_elements = f.tellg() / sizeof(float);
    f.seekg(0, std::ios::beg);
    std::vector<float> buf(num_elements);
    f.read(reinterpret_cast<char*>(buf.data()), num_elements * sizeof(float));
    return buf;
}

static void fill(pcl::PointCloud<pcl::PointXYZI>::Ptr& cloud, const std::vector<float>& d) {
    for (size_t i = 0; i + 5 <= d.size(); i += 5) {
        pcl::PointXYZI p;
        p.x = d[i];
        p.y = d[i + 1];
        p.z = d[i + 2];
        p.intensity = d[i + 3];
        cloud->push_back(p);
    }
}

int main(int argc, char** argv) {
    if (argc < 3) {
        std::fprintf(stderr, "usage: %s src.bin tgt.bin [max_iterations]\n", argv[0]);
        return 2;
    }
    pcl::PointCloud<pcl::PointXYZI>::Ptr cloud_src_in(new pcl::PointCloud<pcl::PointXYZI>);
    pcl::PointCloud<pcl::PointXYZI>::Ptr cloud_tar_in(new pcl::PointCloud<pcl::PointXYZI>);
    pcl::PointCloud<pcl::PointXYZI>::Ptr Final(new pcl::PointCloud<pcl::PointXYZI>);
    fill(cloud_src_in, read_radar_data(argv[1]));
    fill(cloud_tar_in, read_radar_data(argv[2]));

    // ---- the node's call sequence (:510-521) ----
    pcl::IterativeClosestPoint<pcl::PointXYZI, pcl::PointXYZI> icp;
    icp.setInputSource(cloud_src_in);
    icp.setInputTarget(cloud_tar_in);
    if (argc > 3) icp.setMaximumIterations(std::atoi(argv[3]));  // commented out at :513 in the node
    icp.align(*Final);
    std::cout << "has converged:" << icp.hasConverged() << " score: " << icp.getFitnessScore() << std::endl;
    std::cout << icp.getFinalTransformation() << std::endl;
    double score = icp.getFitnessScore();
    Eigen::Matrix<double, 4, 4> icp_result = icp.getFinalTransformation().cast<double>();
    // ---------------------------------------------

    std::printf("RESULT converged=%d score=%.17g iterations=%d points=%zu\n", (int)icp.hasConverged(), score,
                icp.getNrIterations(), Final->size());
    std::printf("T");
    for (int r = 0; r < 4; ++r)
        for (int c = 0; c < 4; ++c) std::printf(" %.9g", icp_result(r, c));
    std::printf("\nFINAL0 %.9g %.9g %.9g %.9g\n", Final->points[0].x, Final->points[0].y, Final->points[0].z,
                Final->points[0].intensity);
    return 0;
}
