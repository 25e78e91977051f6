// icp4radar_replay.cpp — the icp4radar node's frame loop without ROS.
//
// Replays /root/reference/src/iterative_closest_point.cpp:130-820 (USE_BIN_FILES, ICP result mode)
// over a dataset folder and writes the node's output files:
//
//   <dataset>/data/radar_pointcloud_<k>.bin   input, 5-float records (:303-321, read_radar_data :64-82)
//   <dataset>/radar/pcl_info.txt              points per frame (:182-185, :325)
//   <dataset>/radar/velocity.txt              Vxyz per frame, precision 15 (:150-168, :757-765)
//   <dataset>/radar/icp.txt                   R row-major + t per frame, precision 15 (:170-174, :767-791)
//   <dataset>/radar/icp_map.txt               empty (USE_LOCAL_MAP is off, :32, :793-812)
//   <csv>                                     output_result.csv (:188-191, :701-706)
//
// Per frame k (curr = scan k, last = scan k-1, or scan 0 for k = 0 — :306-315): parse, radar ego
// velocity of the current scan (icp4r_ego_velocity: fitSineRansac + split + LSQ, :387-431), ICP of
// curr against last with PCL defaults through the pcl::IterativeClosestPoint facade (:505-521), pose
// composition currOdom = currOdom * T, t += Rtrans * dt, Rtrans = Rtrans * dR (:541-556).  ROS topics,
// the 20-frame submap publisher (:577-633) and stdout are not reproduced; the node's RANSAC of the
// previous scan (:465-493) feeds nothing that is written and is skipped.
//
//   icp4radar_replay <dataset_folder> [--csv PATH] [--batch] [--devices D0,D1,...] [--seed S]
//                    [--max-iterations N] [--use-icp-result CSV]
//
// Empty scans (:505 vs :698-699): the node pushes every frame's points onto cloud_src_in /
// cloud_tar_in and clears them only inside `if (cloud_tar_in->size() && cloud_src_in->size())`.
// When either cloud is empty the frame is not registered AND the other cloud keeps its points, so
// the next frame's points are appended to them: after an empty scan k the next registration is
// scan k+1 against scan k-1 (the tar cloud carried over), and an empty first scan makes frame 2
// register scan 1 + scan 2 against scan 1.  Reproduced here (both modes), as is the node's
// output_time, which advances on registered frames only.
//
// --use-icp-result CSV: the node built with USE_ICP_RESULT (:192-206, :523-540) — no ICP; each
// registered frame takes its transform from the next row of a previous run's output_result.csv.
// The header line is consumed as `firstline` (19 getline(',') + getline('\n'), atof each field);
// a row past the end of the file reads as zeros (getline fails, `value` is empty, atof("") = 0).
// The node fills icp_result(i, j) = data(4*i + j + 1, 1) on a 20x1 vector: column 1 does not exist
// (Eigen's assertion aborts the node's -g build; without assertions it reads past the vector).
// Column 0 — csv field 4*i + j + 1, i.e. Rtrans(i, j) as the non-USE_ICP_RESULT run wrote it — is
// the only defined reading and the one used.  No CSV is written in this mode (:700-707).
//
// --batch: every frame's ICP is independent of the poses (identity guess), so all frames are
// registered in ONE device batch (icp4r_align_batch_host) and composed afterwards — identical output
// to the per-frame loop (the batch path is bit-identical to single calls), one launch sequence.
// --devices D0,D1,... (with --batch): the batch sharded over those devices — one context each,
// contiguous blocks of frames, all shards at once (icp4r_align_batch_multi, include/icp4r/icp4r_multi.h);
// the output is byte-identical to the one-device batch.
#include <sys/stat.h>

#include <array>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <iomanip>
#include <iostream>
#include <memory>
#include <sstream>
#include <string>
#include <vector>

#include "icp4r/icp4r.h"
#include "icp4r/icp4r_ego.h"
#include "icp4r/icp4r_multi.h"
#include "icp4r/pcl_compat.hpp"

namespace {

// read_radar_data (:64-82): the whole file as float32; a missing file is an empty scan.
std::vector<float> read_radar_data(const std::string& path) {
    std::ifstream f(path, std::ifstream::in | std::ifstream::binary);
    if (!f) return {};
    f.seekg(0, std::ios::end);
    const size_t num_elements = (size_t)f.tellg() / sizeof(float);
    f.seekg(0, std::ios::beg);
    std::vector<float> buf(num_elements);
    if (num_elements) f.read(reinterpret_cast<char*>(buf.data()), (std::streamsize)(num_elements * sizeof(float)));
    return buf;
}

bool exists(const std::string& p) {
    struct stat st;
    return stat(p.c_str(), &st) == 0;
}

std::string scan_path(const std::string& folder, size_t k) {
    std::stringstream s;
    s << folder << "data/" << "radar_pointcloud_" << k << ".bin";
    return s.str();
}

// Eigen-like 3x3 / 4x4 double helpers (row-major storage here; the arithmetic is Eigen's
// coefficient order for fixed-size products: sum over k in order).
struct M3 {
    double a[9];
};
struct M4 {
    double a[16];
};
M4 mul4(const M4& A, const M4& B) {
    M4 C;
    for (int i = 0; i < 4; ++i)
        for (int j = 0; j < 4; ++j) {
            double s = A.a[4 * i] * B.a[j];
            for (int k = 1; k < 4; ++k) s += A.a[4 * i + k] * B.a[4 * k + j];
            C.a[4 * i + j] = s;
        }
    return C;
}
M3 mul3(const M3& A, const M3& B) {
    M3 C;
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j) {
            double s = A.a[3 * i] * B.a[j];
            for (int k = 1; k < 3; ++k) s += A.a[3 * i + k] * B.a[3 * k + j];
            C.a[3 * i + j] = s;
        }
    return C;
}

struct FrameOut {
    bool registered = false;
    double T[16];  // icp_result, row-major (double of the float Matrix4f)
    double score = 0;
    double A = 0, b = 0;
    double V[3] = {0, 0, 0};
};

int usage() {
    std::fprintf(stderr, "usage: icp4radar_replay <dataset_folder> [--csv PATH] [--batch] [--devices D0,D1,...] [--seed S] "
                         "[--max-iterations N] [--use-icp-result CSV]\n");
    return 2;
}

}  // namespace

int main(int argc, char** argv) {
    if (argc < 2) return usage();
    std::string dataset_folder = argv[1];
    if (dataset_folder.empty() || dataset_folder.back() != '/') dataset_folder += "/";
    std::string csv = dataset_folder + "output_result.csv";
    bool batch = false;
    std::vector<int> devices;  // --devices: the batch sharded over these (icp4r_align_batch_multi)
    icp4r_ego_params ep;
    icp4r_ego_params_default(&ep);
    int max_iterations = -1;  // PCL default (10) unless given
    std::string icp_result_csv;
    for (int i = 2; i < argc; ++i) {
        if (!std::strcmp(argv[i], "--csv") && i + 1 < argc) csv = argv[++i];
        else if (!std::strcmp(argv[i], "--batch")) batch = true;
        else if (!std::strcmp(argv[i], "--devices") && i + 1 < argc) {
            devices.clear();
            for (const char* c = argv[++i]; *c;) {
                char* end = nullptr;
                devices.push_back((int)std::strtol(c, &end, 10));
                if (end == c) return usage();
                c = *end == ',' ? end + 1 : end;
            }
        }
        else if (!std::strcmp(argv[i], "--seed") && i + 1 < argc) ep.seed = std::strtoull(argv[++i], nullptr, 0);
        else if (!std::strcmp(argv[i], "--max-iterations") && i + 1 < argc) max_iterations = std::atoi(argv[++i]);
        else if (!std::strcmp(argv[i], "--use-icp-result") && i + 1 < argc) icp_result_csv = argv[++i];
        else return usage();
    }
    const bool use_icp_result = !icp_result_csv.empty();
    const std::string out_dir = dataset_folder + "radar";
    if (!exists(out_dir) && mkdir(out_dir.c_str(), 0755) != 0) {  // the node shells out to `sudo mkdir` (:151-156)
        std::perror("mkdir");
        return 1;
    }
    icp4r_ctx* ctx = icp4r::thread_context();

    // ---- the frame loop (:263-721): scans k = 0, 1, ... while radar_pointcloud_<k+1>.bin exists
    std::vector<std::vector<float>> scans;
    for (size_t order = 0;; ++order) {
        scans.push_back(read_radar_data(scan_path(dataset_folder, order)));
        if (!exists(scan_path(dataset_folder, order + 1))) break;
    }
    const size_t nframes = scans.size();
    std::vector<FrameOut> out(nframes);
    std::ofstream pcl_info(out_dir + "/pcl_info.txt", std::ios::trunc);
    pcl_info.setf(std::ios::dec, std::ios::floatfield);
    using Cloud = pcl::PointCloud<pcl::PointXYZI>;
    auto to_cloud = [](const std::vector<float>& xyzi) {
        Cloud::Ptr c(new Cloud);
        const size_t n = xyzi.size() / 4;
        c->points.reserve(n);
        for (size_t i = 0; i < n; ++i)
            c->push_back(pcl::PointXYZI(xyzi[4 * i], xyzi[4 * i + 1], xyzi[4 * i + 2], xyzi[4 * i + 3]));
        return c;
    };
    icp4r_params ip;
    icp4r_params_default(&ip);
    if (max_iterations >= 0) ip.max_iterations = max_iterations;

    for (size_t k = 0; k < nframes; ++k) {
        const std::vector<float>& curr = scans[k];
        pcl_info << curr.size() / 5.0 << std::endl;
        // radar ego velocity of the current scan (:352-431); frame k draws from seed + (k << 32)
        icp4r_ego_params pk = ep;
        pk.seed = ep.seed + ((uint64_t)k << 32);
        icp4r_ego_result er;
        const int n = (int)(curr.size() / 5);
        if (n == 0) {  // A_src = b_src = 0; Vxyz = (KᵀK)⁻¹ Kᵀ Vr over 0 rows: Eigen's empty products give 0
            out[k].A = out[k].b = 0.0;
            continue;
        }
        int rc = icp4r_ego_velocity(ctx, curr.data(), n, &pk, &er, nullptr, nullptr);
        if (rc != ICP4R_OK && rc != ICP4R_E_EMPTY) {
            std::fprintf(stderr, "icp4r_ego_velocity: %s\n", icp4r_last_error());
            return 1;
        }
        out[k].A = er.A;
        out[k].b = er.b;
        for (int c = 0; c < 3; ++c) out[k].V[c] = er.v[c];
    }

    // ---- which frames register, and on which clouds (:505, :698-699): the points of every frame are
    // appended to the running clouds, which are cleared only after a registration.  Registered pair
    // q = (src records, tgt records) in frame order; the list depends on the scan sizes only.
    struct PairIn {
        size_t frame;
        std::vector<float> src, tgt;  // float4 x, y, z, intensity
    };
    std::vector<PairIn> pairs;
    {
        std::vector<float> acc_src, acc_tgt;
        auto push = [](std::vector<float>& acc, const std::vector<float>& rec) {
            const size_t n = rec.size() / 5;
            for (size_t i = 0; i < n; ++i) acc.insert(acc.end(), &rec[5 * i], &rec[5 * i] + 4);
        };
        for (size_t k = 0; k < nframes; ++k) {
            push(acc_src, scans[k]);
            push(acc_tgt, scans[k ? k - 1 : 0]);
            if (acc_src.empty() || acc_tgt.empty()) continue;  // not registered, not cleared
            pairs.push_back({k, std::move(acc_src), std::move(acc_tgt)});
            acc_src.clear();
            acc_tgt.clear();
        }
    }

    if (use_icp_result) {
        // USE_ICP_RESULT (:192-206, :523-540): transforms from a previous run's CSV, no ICP
        std::ifstream file(icp_result_csv.c_str());
        if (!file) {
            std::fprintf(stderr, "cannot open %s\n", icp_result_csv.c_str());
            return 1;
        }
        std::string value;
        double data[20];
        auto read_row = [&]() {
            for (int i = 0; i < 19; i++) {
                std::getline(file, value, ',');
                data[i] = std::atof(value.c_str());
            }
            std::getline(file, value, '\n');
            data[19] = std::atof(value.c_str());
        };
        read_row();  // firstline: the header
        for (const PairIn& q : pairs) {
            read_row();
            FrameOut& f = out[q.frame];
            f.registered = true;
            for (int i = 0; i < 4; i++)
                for (int j = 0; j < 4; j++) f.T[4 * i + j] = data[4 * i + j + 1];  // data(4*i+j+1, 1): see header
            f.score = 0.0;
        }
    } else if (batch) {
        // every registration in one device batch
        std::vector<float> src, tgt;
        std::vector<int64_t> so, to;
        std::vector<int32_t> sn, tn;
        for (const PairIn& q : pairs) {
            so.push_back((int64_t)src.size() / 4);
            to.push_back((int64_t)tgt.size() / 4);
            sn.push_back((int32_t)(q.src.size() / 4));
            tn.push_back((int32_t)(q.tgt.size() / 4));
            src.insert(src.end(), q.src.begin(), q.src.end());
            tgt.insert(tgt.end(), q.tgt.begin(), q.tgt.end());
        }
        std::vector<icp4r_result> res(pairs.size());
        if (!pairs.empty() && devices.size() > 0) {
            // one context per listed device, frames sharded in contiguous blocks
            std::vector<icp4r_ctx*> ctxs(devices.size(), nullptr);
            int rc = ICP4R_OK;
            for (size_t d = 0; d < devices.size() && rc == ICP4R_OK; ++d) rc = icp4r_create(&ctxs[d], devices[d]);
            if (rc == ICP4R_OK)
                rc = icp4r_align_batch_multi(ctxs.data(), (int32_t)ctxs.size(), src.data(), so.data(), sn.data(),
                                             tgt.data(), to.data(), tn.data(), (int32_t)pairs.size(), nullptr, &ip,
                                             res.data());
            if (rc != ICP4R_OK) std::fprintf(stderr, "icp4r_align_batch_multi: %s\n", icp4r_last_error());
            for (icp4r_ctx* c : ctxs) icp4r_destroy(c);
            if (rc != ICP4R_OK) return 1;
        } else if (!pairs.empty()) {
            int rc = icp4r_align_batch_host(ctx, src.data(), so.data(), sn.data(), tgt.data(), to.data(), tn.data(),
                                            (int32_t)pairs.size(), nullptr, &ip, res.data());
            if (rc != ICP4R_OK) {
                std::fprintf(stderr, "icp4r_align_batch_host: %s\n", icp4r_last_error());
                return 1;
            }
        }
        for (size_t q = 0; q < pairs.size(); ++q) {
            FrameOut& f = out[pairs[q].frame];
            f.registered = true;
            for (int r = 0; r < 4; ++r)
                for (int c = 0; c < 4; ++c) f.T[4 * r + c] = (double)res[q].T[4 * c + r];  // column-major float
            f.score = res[q].fitness;
        }
    } else {
        for (const PairIn& q : pairs) {
            auto cloud_src_in = to_cloud(q.src);
            auto cloud_tar_in = to_cloud(q.tgt);
            Cloud Final;
            pcl::IterativeClosestPoint<pcl::PointXYZI, pcl::PointXYZI> icp;  // :510-521
            icp.setInputSource(cloud_src_in);
            icp.setInputTarget(cloud_tar_in);
            if (max_iterations >= 0) icp.setMaximumIterations(max_iterations);
            icp.align(Final);
            const double score = icp.getFitnessScore();
            const Eigen::Matrix4d icp_result = icp.getFinalTransformation().cast<double>();
            FrameOut& f = out[q.frame];
            f.registered = true;
            for (int r = 0; r < 4; ++r)
                for (int c = 0; c < 4; ++c) f.T[4 * r + c] = icp_result(r, c);
            f.score = score;
        }
    }

    // ---- pose composition and the per-frame CSV (:541-558, :701-708)
    FILE* fp = use_icp_result ? nullptr : std::fopen(csv.c_str(), "w+");  // #ifndef USE_ICP_RESULT (:187-191)
    if (!use_icp_result && !fp) {
        std::perror("output_result.csv");
        return 1;
    }
    if (fp) std::fprintf(fp, "#time(s),Rtrans00,Rtrans01,Rtrans02,Rtrans03,Rtrans10,Rtrans11,Rtrans12,Rtrans13,Rtrans20,"
                     "Rtrans21,Rtrans22,Rtrans23,Rtrans00,Rtrans00,Rtrans00,Rtrans00,score,A,b\n");
    M4 currOdom = {{1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1}};
    M3 Rtrans = {{1, 0, 0, 0, 1, 0, 0, 0, 1}};
    double t[3] = {0, 0, 0};
    double output_time = 0;
    std::vector<M3> Icp_Rtrans_result;
    std::vector<std::array<double, 3>> Icp_Ttrans_result;
    for (size_t k = 0; k < nframes; ++k) {
        const FrameOut& f = out[k];
        if (!f.registered) continue;
        M4 T;
        std::memcpy(T.a, f.T, sizeof(T.a));
        M3 dR = {{T.a[0], T.a[1], T.a[2], T.a[4], T.a[5], T.a[6], T.a[8], T.a[9], T.a[10]}};
        const double dt[3] = {T.a[3], T.a[7], T.a[11]};
        Icp_Rtrans_result.push_back(dR);
        Icp_Ttrans_result.push_back({dt[0], dt[1], dt[2]});
        currOdom = mul4(currOdom, T);
        for (int r = 0; r < 3; ++r) {  // t = t + Rtrans * odom_Ptrans
            double s = Rtrans.a[3 * r] * dt[0];
            s += Rtrans.a[3 * r + 1] * dt[1];
            s += Rtrans.a[3 * r + 2] * dt[2];
            t[r] = t[r] + s;
        }
        Rtrans = mul3(Rtrans, dR);
        if (fp) std::fprintf(fp, "%f,%f,%f,%f,%f,%f,%f,%f,%f,%f,%f,%f,%f,%f,%f,%f,%f,%f,%f,%f\n", output_time, T.a[0], T.a[1],
                     T.a[2], T.a[3], T.a[4], T.a[5], T.a[6], T.a[7], T.a[8], T.a[9], T.a[10], T.a[11], T.a[12],
                     T.a[13], T.a[14], T.a[15], f.score, f.A, f.b);
        output_time += 1.0;
    }
    if (fp) std::fclose(fp);

    // ---- the files written after the loop (:757-816)
    std::ofstream velocity_odom(out_dir + "/velocity.txt", std::ios::trunc);
    velocity_odom.setf(std::ios::dec, std::ios::floatfield);
    velocity_odom.precision(15);
    for (size_t k = 0; k < nframes; ++k)
        velocity_odom << out[k].V[0] << ' ' << out[k].V[1] << ' ' << out[k].V[2] << std::endl;
    std::ofstream icp_odom(out_dir + "/icp.txt", std::ios::trunc);
    icp_odom.setf(std::ios::dec, std::ios::floatfield);
    icp_odom.precision(15);
    for (size_t i = 0; i < Icp_Rtrans_result.size(); ++i) {
        const M3& R = Icp_Rtrans_result[i];
        const auto& T = Icp_Ttrans_result[i];
        icp_odom << R.a[0] << ' ' << R.a[1] << ' ' << R.a[2] << ' ' << T[0] << ' ' << R.a[3] << ' ' << R.a[4] << ' '
                 << R.a[5] << ' ' << T[1] << ' ' << R.a[6] << ' ' << R.a[7] << ' ' << R.a[8] << ' ' << T[2]
                 << std::endl;
    }
    std::ofstream icp_map(out_dir + "/icp_map.txt", std::ios::trunc);  // USE_LOCAL_MAP off: stays empty
    std::printf("replayed %zu frames (%zu registered)%s; final position %.6f %.6f %.6f\n", nframes,
                Icp_Rtrans_result.size(), batch ? " in one device batch" : "", t[0], t[1], t[2]);
    return 0;
}
