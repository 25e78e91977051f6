// pcl_compat.hpp — header-only C++ facade: pcl::IterativeClosestPoint over the icp4r C ABI.
//
// Drop-in for the call block at /root/reference/src/iterative_closest_point.cpp:510-521 (and the
// getters radar_odometry.cpp:399-412 consumes).  A maintainer replaces
//     #include <pcl/registration/icp.h>
// by
//     #include <icp4r/pcl_compat.hpp>
// and links libicp4r.so; the call sites stay textually unchanged.
//
// With real PCL and Eigen on the include path their PointCloud / Matrix4f types are used; this image
// has neither, so minimal stand-ins with the same member names are provided (ICP4R_STANDALONE).
// The ICP4R_HAVE_PCL branch stores PCL's own PointCloud<T>::ConstPtr (boost::shared_ptr in PCL 1.8);
// tests/test_facades_pcl18.py compiles it against a PCL-1.8-shaped include tree (tests/cpp/pcl18).
// Define ICP4R_NO_PCL_ALIAS to get icp4r::IterativeClosestPoint without the pcl:: alias.
#pragma once

#include <cfloat>
#include <cstdio>
#include <memory>
#include <stdexcept>
#include <vector>

#include "icp4r/icp4r.h"

#if __has_include(<pcl/point_cloud.h>) && __has_include(<pcl/point_types.h>) && __has_include(<Eigen/Core>)
#include <Eigen/Core>
#include <pcl/point_cloud.h>
#include <pcl/point_types.h>
#define ICP4R_HAVE_PCL 1
#else
#define ICP4R_STANDALONE 1
#include <cstddef>
#include <ostream>

namespace Eigen {
// Column-major fixed-size matrix with the members the reference's call block uses.
template <typename Scalar, int Rows, int Cols>
struct Matrix {
    Scalar m[Rows * Cols] = {};
    Scalar& operator()(int r, int c) { return m[c * Rows + r]; }
    const Scalar& operator()(int r, int c) const { return m[c * Rows + r]; }
    Scalar* data() { return m; }
    const Scalar* data() const { return m; }
    static Matrix Identity() {
        Matrix I;
        for (int k = 0; k < Rows && k < Cols; ++k) I(k, k) = Scalar(1);
        return I;
    }
    template <typename T>
    Matrix<T, Rows, Cols> cast() const {
        Matrix<T, Rows, Cols> o;
        for (int k = 0; k < Rows * Cols; ++k) o.m[k] = static_cast<T>(m[k]);
        return o;
    }
    bool operator!=(const Matrix& o) const {
        for (int k = 0; k < Rows * Cols; ++k)
            if (m[k] != o.m[k]) return true;
        return false;
    }
};
using Matrix4f = Matrix<float, 4, 4>;
using Matrix4d = Matrix<double, 4, 4>;

template <typename S, int R, int C>
std::ostream& operator<<(std::ostream& os, const Matrix<S, R, C>& a) {
    for (int r = 0; r < R; ++r) {
        for (int c = 0; c < C; ++c) os << (c ? " " : "") << a(r, c);
        if (r + 1 < R) os << "\n";
    }
    return os;
}
}  // namespace Eigen

namespace pcl {
// pcl::PointXYZI memory layout (PCL_ADD_POINT4D + intensity union): 32 bytes, 16-aligned.
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
    PointXYZI(float x_, float y_, float z_, float i_) : data{x_, y_, z_, 1.f}, data_c{i_, 0.f, 0.f, 0.f} {}
};
static_assert(sizeof(PointXYZI) == 32, "PointXYZI must match PCL's 32-byte layout");

template <typename PointT>
class PointCloud {
  public:
    using Ptr = std::shared_ptr<PointCloud<PointT>>;
    using ConstPtr = std::shared_ptr<const PointCloud<PointT>>;
    std::vector<PointT> points;
    size_t size() const { return points.size(); }
    bool empty() const { return points.empty(); }
    void push_back(const PointT& p) { points.push_back(p); }
    void clear() { points.clear(); }
    void resize(size_t n) { points.resize(n); }
    PointT& operator[](size_t i) { return points[i]; }
    const PointT& operator[](size_t i) const { return points[i]; }
};
}  // namespace pcl
#endif

namespace icp4r {

// One context per host thread (PCL objects are not thread-safe either; calls are serialized).
inline icp4r_ctx* thread_context() {
    struct Holder {
        icp4r_ctx* ctx = nullptr;
        ~Holder() {
            if (ctx) icp4r_destroy(ctx);
        }
    };
    thread_local Holder h;
    if (!h.ctx) {
        int rc = icp4r_create(&h.ctx, 0);
        if (rc != ICP4R_OK) throw std::runtime_error(std::string("icp4r_create: ") + icp4r_last_error());
    }
    return h.ctx;
}

// pcl::IterativeClosestPoint<PointSource, PointTarget, float> with PCL 1.8.1 defaults.
template <typename PointSource, typename PointTarget, typename Scalar = float>
class IterativeClosestPoint {
  public:
    using PointCloudSource = pcl::PointCloud<PointSource>;
    using PointCloudTarget = pcl::PointCloud<PointTarget>;
    // PCL's own pointer types: boost::shared_ptr in PCL 1.8 (the node's ROS melodic), std::shared_ptr
    // from PCL 1.11 and in the stand-ins above — the caller's Ptr converts to ConstPtr either way
    using PointCloudSourceConstPtr = typename PointCloudSource::ConstPtr;
    using PointCloudTargetConstPtr = typename PointCloudTarget::ConstPtr;
    using Matrix4 = Eigen::Matrix<Scalar, 4, 4>;

    IterativeClosestPoint() { icp4r_params_default(&params_); }

    // Registration::setInputSource / setInputTarget (const PointCloud::ConstPtr&), no copy
    void setInputSource(const PointCloudSourceConstPtr& cloud) { src_ = cloud; }
    void setInputTarget(const PointCloudTargetConstPtr& cloud) { tgt_ = cloud; }
    PointCloudSourceConstPtr const getInputSource() { return src_; }
    PointCloudTargetConstPtr const getInputTarget() { return tgt_; }

    void setMaximumIterations(int nr_iterations) { params_.max_iterations = nr_iterations; }
    int getMaximumIterations() const { return params_.max_iterations; }
    void setMaxCorrespondenceDistance(double d) { params_.max_correspondence_distance = d; }
    double getMaxCorrespondenceDistance() const { return params_.max_correspondence_distance; }
    void setTransformationEpsilon(double e) { params_.transformation_epsilon = e; }
    double getTransformationEpsilon() const { return params_.transformation_epsilon; }
    void setTransformationRotationEpsilon(double e) { params_.transformation_rotation_epsilon = e; }
    void setEuclideanFitnessEpsilon(double e) { params_.euclidean_fitness_epsilon = e; }
    double getEuclideanFitnessEpsilon() const { return params_.euclidean_fitness_epsilon; }
    // build extensions (no PCL counterpart)
    void setHuberDelta(double delta) { params_.huber_delta = delta; }
    void setNumerics(icp4r_numerics n) { params_.numerics = n; }

    // Registration::align(output) / align(output, guess)
    void align(PointCloudSource& output) { align_impl(output, nullptr); }
    void align(PointCloudSource& output, const Matrix4& guess) { align_impl(output, &guess); }

    bool hasConverged() const { return converged_; }
    Matrix4 getFinalTransformation() const { return final_; }
    int getNrIterations() const { return result_.iterations; }
    int getStatus() const { return result_.status; }

    // Registration::getFitnessScore(max_range = DBL_MAX)
    double getFitnessScore(double max_range = DBL_MAX) {
        if (!src_ || !tgt_) return DBL_MAX;
        if (max_range == params_.fitness_max_range && have_result_) return result_.fitness;
        double f = DBL_MAX;
        icp4r_fitness(thread_context(), ptr(*src_), (int32_t)src_->size(), (int32_t)sizeof(PointSource), ptr(*tgt_),
                      (int32_t)tgt_->size(), (int32_t)sizeof(PointTarget), final_.data(), max_range, &f);
        return f;
    }

  private:
    template <typename Cloud>
    static const float* ptr(const Cloud& c) {
        return c.points.empty() ? nullptr : reinterpret_cast<const float*>(&c.points[0]);
    }

    void align_impl(PointCloudSource& output, const Matrix4* guess) {
        converged_ = false;
        have_result_ = false;
        final_ = Matrix4::Identity();
        if (!tgt_) {
            std::fprintf(stderr, "[pcl::IterativeClosestPoint::compute] No input target dataset was given!\n");
            return;
        }
        if (!src_) return;
        const int32_t n = (int32_t)src_->size(), m = (int32_t)tgt_->size();
        std::vector<float> aligned((size_t)(n > 0 ? n : 1) * 4);
        int rc = icp4r_align(thread_context(), ptr(*src_), n, (int32_t)sizeof(PointSource), ptr(*tgt_), m,
                             (int32_t)sizeof(PointTarget), guess ? guess->data() : nullptr, &params_, &result_,
                             aligned.data(), 16);
        if (rc != ICP4R_OK && rc != ICP4R_E_TOO_FEW_CORR && rc != ICP4R_E_EMPTY && rc != ICP4R_E_NONFINITE)
            throw std::runtime_error(std::string("icp4r_align: ") + icp4r_last_error());
        if (rc != ICP4R_OK) std::fprintf(stderr, "[pcl::IterativeClosestPoint::computeTransformation] %s\n", icp4r_last_error());
        have_result_ = true;
        converged_ = result_.converged != 0;
        for (int k = 0; k < 16; ++k) final_.data()[k] = result_.T[k];
        output = *src_;  // output := input, then xyz := final * input (intensity kept)
        for (int32_t i = 0; i < n; ++i) {
            output.points[i].x = aligned[4 * (size_t)i + 0];
            output.points[i].y = aligned[4 * (size_t)i + 1];
            output.points[i].z = aligned[4 * (size_t)i + 2];
        }
    }

    PointCloudSourceConstPtr src_;
    PointCloudTargetConstPtr tgt_;
    icp4r_params params_;
    icp4r_result result_{};
    Matrix4 final_ = Matrix4::Identity();
    bool converged_ = false;
    bool have_result_ = false;
};

}  // namespace icp4r

#ifndef ICP4R_NO_PCL_ALIAS
namespace pcl {
template <typename PointSource, typename PointTarget, typename Scalar = float>
using IterativeClosestPoint = icp4r::IterativeClosestPoint<PointSource, PointTarget, Scalar>;
}
#endif
