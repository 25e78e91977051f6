// radar_odometry's map calls (src/radar_odometry.cpp:92, :343-348, :382-396) compiled against
// include/icp4r/ikd_compat.hpp instead of ikd_Tree.h.  Scans come from two .bin files (the node's
// record format); the first builds the map in the radar frame (:347), the second is associated to
// the world with the pose given on the command line (the node's pointAssociateToMap, :137-145) and
// added (:390); then Sector_Search(p_now, RADAR_RADIUS, heading) (:396).  Prints the submap for
// tests/test_map.py to compare with the oracle.
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <fstream>
#include <vector>

#include "icp4r/ikd_compat.hpp"

#define RADAR_RADIUS 80  // radar_odometry.cpp:36

typedef pcl::PointXYZI PointType;
KD_TREE<pcl::PointXYZI> ikd_Tree(0.3, 0.6, 0.5);  // radar_odometry.cpp:92, namespace scope as there

static double Rtrans[9], t_w_curr[3];

// radar_odometry.cpp:137-145 (Eigen: Rtrans * point_curr + t_w_curr, double, per row in order)
static void pointAssociateToMap(PointType const* const pi, PointType* const po) {
    double w[3];
    for (int r = 0; r < 3; ++r) {
        double s = Rtrans[3 * r] * (double)pi->x;
        s = s + Rtrans[3 * r + 1] * (double)pi->y;
        s = s + Rtrans[3 * r + 2] * (double)pi->z;
        w[r] = s + t_w_curr[r];
    }
    po->x = (float)w[0];
    po->y = (float)w[1];
    po->z = (float)w[2];
    po->intensity = pi->intensity;
}

static pcl::PointCloud<PointType>::Ptr read_scan(const char* path) {
    pcl::PointCloud<PointType>::Ptr c(new pcl::PointCloud<PointType>);
    std::ifstream f(path, std::ios::binary);
    float rec[5];
    while (f.read(reinterpret_cast<char*>(rec), sizeof(rec))) {
        PointType p;
        p.x = rec[0];
        p.y = rec[1];
        p.z = rec[2];
        p.intensity = rec[3];
        c->push_back(p);
    }
    return c;
}

int main(int argc, char** argv) {
    if (argc < 6) {
        std::fprintf(stderr, "usage: %s first.bin next.bin x y yaw_deg\n", argv[0]);
        return 2;
    }
    pcl::PointCloud<PointType>::Ptr src = read_scan(argv[1]);
    ikd_Tree.Build(src->points);  // :347
    ikd_Tree.set_downsample_param(0.5);  // :348
    const double x = atof(argv[3]), y = atof(argv[4]), yaw = atof(argv[5]) * M_PI / 180.0;
    const double R[9] = {cos(yaw), -sin(yaw), 0, sin(yaw), cos(yaw), 0, 0, 0, 1};
    for (int k = 0; k < 9; ++k) Rtrans[k] = R[k];
    t_w_curr[0] = x;
    t_w_curr[1] = y;
    t_w_curr[2] = 0;
    pcl::PointCloud<PointType>::Ptr next = read_scan(argv[2]);
    pcl::PointCloud<PointType>::Ptr scan_map(new pcl::PointCloud<PointType>);
    pcl::PointCloud<PointType>::Ptr SubMap(new pcl::PointCloud<PointType>);
    PointType p_sel;
    for (size_t i = 0; i < next->size(); i++) {  // :384-389
        pointAssociateToMap(&next->points[i], &p_sel);
        scan_map->push_back(p_sel);
    }
    ikd_Tree.Add_Points(scan_map->points, false);  // :390
    PointType p_now;
    p_now.x = (float)x;
    p_now.y = (float)y;
    p_now.z = 0;
    const double heading = atof(argv[5]);
    ikd_Tree.Sector_Search(p_now, RADAR_RADIUS, heading, SubMap->points);  // :396
    std::printf("map %d submap %zu\n", ikd_Tree.size(), SubMap->size());
    for (size_t i = 0; i < SubMap->size(); ++i)
        std::printf("%.9g %.9g %.9g %.9g\n", SubMap->points[i].x, SubMap->points[i].y, SubMap->points[i].z,
                    SubMap->points[i].intensity);
    return 0;
}
