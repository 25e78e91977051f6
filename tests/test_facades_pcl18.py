"""The C++ facades against PCL 1.8's types, on CPU (compile + link only; no GPU call).

PCL 1.8.1 (ROS melodic, the node's platform) hands clouds around as boost::shared_ptr
(`iterative_closest_point.cpp:220-222`, used at `:511-512`; `radar_odometry.cpp:86-91`, used at
`:402-403`).  tests/cpp/pcl18 is a PCL-1.8-shaped include tree (boost::shared_ptr that is not a
std::shared_ptr, aligned-allocator point vectors, Eigen expression return types): the call-site
programs compile unchanged against it, through the facades' ICP4R_HAVE_PCL branches, and
pcl18_check.cpp asserts those branches store PCL's own ConstPtr.  The -m gpu tests run the
resulting programs and compare them with the oracle."""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CPP = os.path.join(ROOT, "tests", "cpp")
LIB = os.path.join(ROOT, "icp-4dradar_amd", "icp4r", "_lib")


def _compile(src, out, extra=()):
    cmd = ["g++", "-O1", "-std=c++17", "-Wall", "-Werror", f"-I{CPP}/pcl18", f"-I{ROOT}/include", *extra, "-o", str(out),
           os.path.join(CPP, src), f"-L{LIB}", "-licp4r", f"-Wl,-rpath,{LIB}"]
    return subprocess.run(cmd, capture_output=True, text=True, timeout=300)


@pytest.mark.parametrize("src", ["callsite.cpp", "map_callsite.cpp", "gicp_callsite.cpp", "pcl18_check.cpp"])
def test_facade_compiles_against_pcl18_tree(src, tmp_path):
    r = _compile(src, tmp_path / "a.out")
    assert r.returncode == 0, r.stderr[-4000:]


def test_pcl18_check_runs(tmp_path):
    """pcl18_check only sets inputs (no device call): Ptr -> ConstPtr stored without a copy."""
    r = _compile("pcl18_check.cpp", tmp_path / "chk")
    assert r.returncode == 0, r.stderr[-4000:]
    assert subprocess.run([str(tmp_path / "chk")], timeout=60).returncode == 0


def test_std_shared_ptr_storage_would_not_compile(tmp_path):
    """The stand-in is strict enough to catch the round-1 facade: storing the caller's PCL 1.8 cloud
    pointer in a std::shared_ptr does not compile."""
    src = tmp_path / "neg.cpp"
    src.write_text('#include <memory>\n#include <pcl/point_cloud.h>\n#include <pcl/point_types.h>\n'
                   'int main() { pcl::PointCloud<pcl::PointXYZI>::Ptr p(new pcl::PointCloud<pcl::PointXYZI>);\n'
                   '  std::shared_ptr<const pcl::PointCloud<pcl::PointXYZI>> s = p; return s ? 0 : 1; }\n')
    r = subprocess.run(["g++", "-std=c++17", f"-I{CPP}/pcl18", "-c", "-o", str(tmp_path / "neg.o"), str(src)],
                       capture_output=True, text=True, timeout=120)
    assert r.returncode != 0
