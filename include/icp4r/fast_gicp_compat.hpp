// fast_gicp_compat.hpp — header-only C++ facade: fast_gicp::FastGICPSingleThread over the icp4r
// generalized-ICP C ABI (include/icp4r/icp4r_gicp.h).
//
// Drop-in for the call block at /root/reference/src/radar_odometry.cpp:399-411:
//     fast_gicp::FastGICPSingleThread<pcl::PointXYZI, pcl::PointXYZI> fgicp_st;
//     fgicp_st.clearTarget(); fgicp_st.clearSource();
//     fgicp_st.setInputTarget(SubMap); fgicp_st.setInputSource(scan_map);
//     fgicp_st.setCorrespondenceRandomness(5);
//     fgicp_st.align(*Final);
//     fgicp_st.getFitnessScore(); fgicp_st.hasConverged(); fgicp_st.getFinalTransformation();
// A maintainer replaces
//     #include <fast_gicp/gicp/fast_gicp.hpp>
//     #include <fast_gicp/gicp/fast_gicp_st.hpp>      (radar_odometry.cpp:31-32)
// by
//     #include <icp4r/fast_gicp_compat.hpp>
// and links libicp4r.so.  The defaults are fast_gicp's (k = 20, PLANE regularisation, 64 iterations,
// rotation / transformation epsilon 2e-3 / 5e-4, LM with lambda factor 1e-9).  Errors follow the
// PCL convention the reference relies on: nothing throws on bad input, hasConverged() is false.
#pragma once

#include <cfloat>
#include <cstdio>
#include <memory>
#include <stdexcept>
#include <string>
#include <vector>

#include "icp4r/icp4r_gicp.h"
#include "icp4r/pcl_compat.hpp"

namespace fast_gicp {

// fast_gicp::RegularizationMethod
enum class RegularizationMethod { NONE = 0, MIN_EIG = 1, NORMALIZE_MIN_EIG = 2, PLANE = 3, FROBENIUS = 4 };

template <typename PointSource, typename PointTarget>
class FastGICPSingleThread {
  public:
    using PointCloudSource = pcl::PointCloud<PointSource>;
    using PointCloudTarget = pcl::PointCloud<PointTarget>;
    using PointCloudSourceConstPtr = typename PointCloudSource::ConstPtr;  // boost::shared_ptr in PCL 1.8
    using PointCloudTargetConstPtr = typename PointCloudTarget::ConstPtr;
    using Matrix4 = Eigen::Matrix<float, 4, 4>;

    FastGICPSingleThread() { icp4r_gicp_params_default(&params_); }

    void clearSource() { src_.reset(); }
    void clearTarget() { tgt_.reset(); }
    void setInputSource(const PointCloudSourceConstPtr& cloud) { src_ = cloud; }
    void setInputTarget(const PointCloudTargetConstPtr& cloud) { tgt_ = cloud; }

    void setCorrespondenceRandomness(int k) { params_.k_correspondences = k; }
    void setRegularizationMethod(RegularizationMethod m) { params_.regularization = (int32_t)m; }
    void setMaxCorrespondenceDistance(double d) { params_.max_correspondence_distance = d; }
    void setMaximumIterations(int n) { params_.max_iterations = n; }
    void setRotationEpsilon(double e) { params_.rotation_epsilon = e; }
    void setTransformationEpsilon(double e) { params_.transformation_epsilon = e; }
    void setInitialLambdaFactor(double f) { params_.lm_init_lambda_factor = f; }
    void setMaxLMIterations(int n) { params_.lm_max_iterations = n; }

    // Registration::align(output) / align(output, guess)
    void align(PointCloudSource& output) { align_impl(output, nullptr); }
    void align(PointCloudSource& output, const Matrix4& guess) { align_impl(output, &guess); }

    bool hasConverged() const { return converged_; }
    Matrix4 getFinalTransformation() const { return final_; }
    int getNrIterations() const { return result_.iterations; }  // fast_gicp's nr_iterations_ (last index)
    // Registration::getFitnessScore(DBL_MAX): computed once inside align (params.compute_fitness)
    double getFitnessScore(double max_range = DBL_MAX) {
        if (!have_result_) return DBL_MAX;
        if (max_range == DBL_MAX) return result_.fitness;
        double f = DBL_MAX;
        icp4r_fitness(icp4r::thread_context(), ptr(*src_), (int32_t)src_->size(), (int32_t)sizeof(PointSource),
                      ptr(*tgt_), (int32_t)tgt_->size(), (int32_t)sizeof(PointTarget), final_.data(), max_range, &f);
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
        if (!src_ || !tgt_) {
            std::fprintf(stderr, "[fast_gicp::align] source or target not set\n");
            return;
        }
        const int32_t n = (int32_t)src_->size(), m = (int32_t)tgt_->size();
        std::vector<float> aligned((size_t)(n > 0 ? n : 1) * 4);
        params_.compute_fitness = 1;
        const int rc = icp4r_gicp_align(icp4r::thread_context(), ptr(*src_), n, (int32_t)sizeof(PointSource), ptr(*tgt_),
                                        m, (int32_t)sizeof(PointTarget), guess ? guess->data() : nullptr, &params_,
                                        &result_, aligned.data(), 16);
        if (rc != ICP4R_OK && rc != ICP4R_E_EMPTY && rc != ICP4R_E_NONFINITE && rc != ICP4R_E_TOO_FEW_CORR)
            throw std::runtime_error(std::string("icp4r_gicp_align: ") + icp4r_last_error());
        if (rc != ICP4R_OK) {
            std::fprintf(stderr, "[fast_gicp::align] %s\n", icp4r_last_error());
            return;
        }
        have_result_ = true;
        converged_ = result_.converged != 0;
        for (int k = 0; k < 16; ++k) final_.data()[k] = result_.T[k];
        output = *src_;  // pcl::transformPointCloud(*input_, output, final_transformation_), intensity kept
        for (int32_t i = 0; i < n; ++i) {
            output.points[i].x = aligned[4 * (size_t)i + 0];
            output.points[i].y = aligned[4 * (size_t)i + 1];
            output.points[i].z = aligned[4 * (size_t)i + 2];
        }
    }

    PointCloudSourceConstPtr src_;
    PointCloudTargetConstPtr tgt_;
    icp4r_gicp_params params_;
    icp4r_result result_{};
    Matrix4 final_ = Matrix4::Identity();
    bool converged_ = false;
    bool have_result_ = false;
};

template <typename PointSource, typename PointTarget>
using FastGICP = FastGICPSingleThread<PointSource, PointTarget>;  // (same single-pair device path)

}  // namespace fast_gicp
