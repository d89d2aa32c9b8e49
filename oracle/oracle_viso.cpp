// TEST INFRASTRUCTURE ONLY — oracle of the whole per-frame path:
// Viso::OnNewFrame (src/viso.cpp:7-145) driving the stage restatements of
// oracle_image.cpp / oracle_track.cpp / oracle_geom.cpp.  Headless: the
// cv::imshow / cv::waitKey / std::cout lines (src/viso.cpp:55-75, 123-135)
// are display only and are not restated.  Copy-free: the reference's
// by-value Map::GetPoints()/Keyframes() copies (include/map.h:18-19) do not
// change results and are not reproduced.
#include <cmath>
#include <cstring>
#include <memory>
#include <vector>

#include "oracle_common.hpp"
#include "oracle_se3.hpp"
#include "viso_oracle.h"

using namespace oracle;

namespace {

struct Frame {
    std::vector<uint8_t> pyr;
    double R[9] = {1, 0, 0, 0, 1, 0, 0, 0, 1};  // Keyframe ctor: R = I, T = 0 (keyframe.h:33-34)
    double T[3] = {0, 0, 0};
    double pose12[12];
    const double* pose() {
        std::memcpy(pose12, R, sizeof(R));
        std::memcpy(pose12 + 9, T, sizeof(T));
        return pose12;
    }
};
using FramePtr = std::shared_ptr<Frame>;

// Eigen 3x3 inverse (compute_inverse<..., 3>): cofactors + 1/det
void eigen_inverse3(const double* m, double* inv) {
    auto M = [&](int i, int j) { return m[3 * i + j]; };
    auto cof = [&](int i, int j) {
        int i1 = (i + 1) % 3, i2 = (i + 2) % 3, j1 = (j + 1) % 3, j2 = (j + 2) % 3;
        return M(i1, j1) * M(i2, j2) - M(i1, j2) * M(i2, j1);
    };
    double c0[3] = {cof(0, 0), cof(1, 0), cof(2, 0)};
    double det = (c0[0] * M(0, 0) + c0[1] * M(1, 0)) + c0[2] * M(2, 0);
    double invdet = 1.0 / det;
    inv[0] = c0[0] * invdet;
    inv[1] = c0[1] * invdet;
    inv[2] = c0[2] * invdet;
    inv[3] = cof(0, 1) * invdet;
    inv[4] = cof(1, 1) * invdet;
    inv[5] = cof(2, 1) * invdet;
    inv[6] = cof(0, 2) * invdet;
    inv[7] = cof(1, 2) * invdet;
    inv[8] = cof(2, 2) * invdet;
}

}  // namespace

struct oracle_viso {
    oracle_params p;
    double K4[4];
    double Kinv[9];
    int state = 0;  // kInitialization
    int w = 0, h = 0;
    FramePtr last_frame, ref_frame;
    std::vector<FramePtr> keyframes;
    std::vector<float> kp1, kp2;  // x,y interleaved (cv::KeyPoint::pt)
    std::vector<uint8_t> success;
    int frame_cnt = 0;  // include/viso.h:38 is uninitialised; treated as 0
    double initR[9] = {1, 0, 0, 0, 1, 0, 0, 0, 1};
    double initT[3] = {0, 0, 0};
    std::vector<double> points;  // map points (world = first keyframe camera)
    std::vector<SE3> poses;
    double stats[16] = {0};
    int frames = 0;
    // last LK alignment
    std::vector<int32_t> al_kf;
    std::vector<uint8_t> al_succ;
    std::vector<double> al_before, al_after;
    // stereo initialisation (viso_set_stereo)
    double stereo_base = 0;
    int max_disp = 0, min_disp = 1;
    // stereo keyframe insertion (viso_set_keyframes; the repo's own map
    // maintenance)
    int kf_interval = 0, kf_permille = 0;
    long long track_cnt = 0;
    // photometric BA after every keyframe insertion (viso_set_bundle_adjust;
    // oracle_ba.cpp): LM iterations (0 = off) and each point's host keyframe
    int ba_iterations = 0;
    std::vector<int32_t> point_host;
};

extern "C" {

void oracle_default_params(oracle_params* p, double fx, double fy, double cx, double cy, int w,
                           int h) {
    std::memset(p, 0, sizeof(*p));
    p->fx = fx;
    p->fy = fy;
    p->cx = cx;
    p->cy = cy;
    p->width = w;
    p->height = h;
    p->reinitialize_after = 10;
    p->fast_thresh = 50;
    p->projection_error_thresh = 0.3;
    p->parallax_thresh = 1.0;
    p->disparity_squared_thresh = 225.0;
    p->photometric_error_thresh = (4.0 * 2) * (4.0 * 2) * 15 * 15;
    p->enable_tracking = 0;
    p->ransac_e_iters = 1000;
    p->ransac_h_iters = 2000;
    p->ransac_confidence = 0.99;
    p->ransac_seed = 0x5eed5eedULL;
}

oracle_viso* oracle_viso_create(const oracle_params* p) {
    oracle_viso* v = new oracle_viso();
    v->p = *p;
    v->K4[0] = p->fx;
    v->K4[1] = p->fy;
    v->K4[2] = p->cx;
    v->K4[3] = p->cy;
    double K[9] = {p->fx, 0, p->cx, 0, p->fy, p->cy, 0, 0, 1};
    eigen_inverse3(K, v->Kinv);
    v->w = p->width;
    v->h = p->height;
    return v;
}

void oracle_viso_destroy(oracle_viso* v) { delete v; }

namespace {
// map creation from one stereo pair (the stereo replacement of
// src/viso.cpp:79-96): returns false when there are <= 50 points
bool stereo_init(oracle_viso* v, const FramePtr& cur, const uint8_t* right) {
    const int w = v->w, h = v->h;
    std::vector<int32_t> xs((size_t)w * h / 4 + 16), ys(xs.size()), sc(xs.size());
    const int n = oracle_fast(cur->pyr.data(), w, h, v->p.fast_thresh, xs.data(), ys.data(), sc.data(),
                              (int)xs.size());
    std::vector<double> pts((size_t)3 * n + 3);
    const int m = oracle_stereo_points(cur->pyr.data(), right, w, h, xs.data(), ys.data(), n, v->max_disp,
                                       v->min_disp, v->K4, v->stereo_base, pts.data());
    v->stats[1] = n;
    v->stats[2] = m;
    if (m <= 50) return false;
    v->keyframes.clear();
    v->keyframes.push_back(cur);
    v->points.assign(pts.begin(), pts.begin() + 3 * (size_t)m);
    v->point_host.assign((size_t)m, 0);
    v->state = v->p.enable_tracking ? 1 : 2;
    v->stats[3] = -2;  // stereo initialisation
    v->stats[12] = 1;
    return true;
}

void on_new(oracle_viso* v, const uint8_t* img, const uint8_t* right) {
    const int w = v->w, h = v->h;
    FramePtr cur = std::make_shared<Frame>();
    cur->pyr.resize(oracle_pyramid_bytes(w, h));
    oracle_pyramid(img, w, h, cur->pyr.data());
    for (int k = 0; k < 16; ++k) v->stats[k] = 0;
    v->stats[12] = 0;
    switch (v->state) {
        case 0: {  // kInitialization
            if (right && v->stereo_base > 0 && stereo_init(v, cur, right)) break;
            if (v->frame_cnt > 0 && v->frame_cnt <= v->p.reinitialize_after) {
                int n = (int)v->kp1.size() / 2;
                v->success.assign((size_t)n, 0);
                oracle_klt(v->ref_frame->pyr.data(), cur->pyr.data(), w, h, v->kp1.data(),
                           v->kp2.data(), v->success.data(), n, v->p.photometric_error_thresh);
                // erase failed tracks (src/viso.cpp:23-40)
                int m = 0;
                for (int i = 0; i < n; ++i)
                    if (v->success[(size_t)i]) {
                        v->kp1[(size_t)2 * m] = v->kp1[(size_t)2 * i];
                        v->kp1[(size_t)2 * m + 1] = v->kp1[(size_t)2 * i + 1];
                        v->kp2[(size_t)2 * m] = v->kp2[(size_t)2 * i];
                        v->kp2[(size_t)2 * m + 1] = v->kp2[(size_t)2 * i + 1];
                        ++m;
                    }
                v->kp1.resize((size_t)2 * m);
                v->kp2.resize((size_t)2 * m);
                v->success.clear();
                std::vector<double> p1((size_t)3 * m), p2((size_t)3 * m);
                const double* Ki = v->Kinv;
                for (int i = 0; i < m; ++i) {
                    const double a[3] = {(double)v->kp1[(size_t)2 * i], (double)v->kp1[(size_t)2 * i + 1], 1};
                    const double b[3] = {(double)v->kp2[(size_t)2 * i], (double)v->kp2[(size_t)2 * i + 1], 1};
                    for (int r = 0; r < 3; ++r) {
                        p1[(size_t)3 * i + r] = Ki[3 * r] * a[0] + Ki[3 * r + 1] * a[1] + Ki[3 * r + 2] * a[2];
                        p2[(size_t)3 * i + r] = Ki[3 * r] * b[0] + Ki[3 * r + 1] * b[1] + Ki[3 * r + 2] * b[2];
                    }
                }
                int nr_inliers = 0;
                std::vector<uint8_t> inl((size_t)m);
                std::vector<double> pts((size_t)3 * m);
                double st[8];
                double R[9], T[3];
                std::memcpy(R, v->initR, sizeof(R));
                std::memcpy(T, v->initT, sizeof(T));
                int ran = oracle_pose_2d2d(p1.data(), p2.data(), m, v->K4, &v->p, R, T, inl.data(),
                                           pts.data(), nullptr, st);
                if (ran) {
                    nr_inliers = (int)st[0];
                    std::memcpy(v->initR, R, sizeof(R));
                    std::memcpy(v->initT, T, sizeof(T));
                    // init_.success = best_inliers (empty when no motion had inliers)
                    if (st[1] >= 0) v->success.assign(inl.begin(), inl.end());
                }
                v->stats[1] = m;
                v->stats[2] = nr_inliers;
                v->stats[3] = ran ? st[1] : -1;
                v->stats[4] = ran ? st[2] : 0;
                v->stats[8] = st[3];
                const double thresh = 0.9;
                if (m > 50 && nr_inliers > 0 && (nr_inliers / (double)m) > thresh) {
                    v->keyframes.clear();
                    v->keyframes.push_back(v->ref_frame);
                    v->keyframes.push_back(cur);
                    std::memcpy(cur->R, v->initR, sizeof(cur->R));
                    std::memcpy(cur->T, v->initT, sizeof(cur->T));
                    v->points.clear();
                    for (int i = 0; i < m; ++i)
                        if (v->success[(size_t)i])
                            for (int k = 0; k < 3; ++k) v->points.push_back(pts[(size_t)3 * i + k]);
                    v->point_host.assign(v->points.size() / 3, 0);  // in keyframe 0's (ref) frame
                    v->state = v->p.enable_tracking ? 1 : 2;  // kRunning : kFinished (src/viso.cpp:97)
                    v->stats[12] = 1;
                    break;
                }
            } else {
                // re-detect (src/viso.cpp:100-108)
                std::vector<int32_t> xs((size_t)w * h / 4 + 16), ys(xs.size()), sc(xs.size());
                int n = oracle_fast(cur->pyr.data(), w, h, v->p.fast_thresh, xs.data(), ys.data(),
                                    sc.data(), (int)xs.size());
                v->kp1.resize((size_t)2 * n);
                for (int i = 0; i < n; ++i) {
                    v->kp1[(size_t)2 * i] = (float)xs[(size_t)i];
                    v->kp1[(size_t)2 * i + 1] = (float)ys[(size_t)i];
                }
                v->kp2 = v->kp1;
                v->success.clear();
                v->ref_frame = cur;
                v->frame_cnt = 0;
                v->stats[1] = n;
            }
            ++v->frame_cnt;
            break;
        }
        case 1: {  // kRunning
            // Sophus::SE3d X(last_frame->GetR(), last_frame->GetT()) (src/viso.cpp:114)
            SE3 X = se3_from_Rt(v->last_frame->R, v->last_frame->T);
            const int np = (int)v->points.size() / 3;
            // DirectPoseEstimationMultiLayer (src/viso.cpp:760-766)
            double st[50];
            for (int level = 3; level >= 0; --level) {
                direct_layer(v->last_frame->pyr.data(), cur->pyr.data(), w, h, v->K4,
                             v->points.data(), np, v->last_frame->pose(), X, level, st);
                if (level == 0) {
                    v->stats[9] = st[0];
                    v->stats[10] = st[1];
                }
            }
            quat_to_matrix(X.q, cur->R);
            std::memcpy(cur->T, X.t, sizeof(cur->T));
            // LKAlignment (src/viso.cpp:768-843)
            const int nk = (int)v->keyframes.size();
            std::vector<const uint8_t*> kp(nk);
            std::vector<double> kpose((size_t)12 * nk);
            for (int j = 0; j < nk; ++j) {
                kp[(size_t)j] = v->keyframes[(size_t)j]->pyr.data();
                std::memcpy(&kpose[(size_t)12 * j], v->keyframes[(size_t)j]->pose(), 12 * sizeof(double));
            }
            v->al_kf.assign((size_t)np, -1);
            v->al_succ.assign((size_t)np, 0);
            v->al_before.assign((size_t)2 * np, 0.0);
            v->al_after.assign((size_t)2 * np, 0.0);
            oracle_lk_align(kp.data(), kpose.data(), nk, cur->pyr.data(), cur->pose(), w, h, v->K4,
                            v->points.data(), np, v->p.photometric_error_thresh, v->al_kf.data(),
                            v->al_succ.data(), v->al_before.data(), v->al_after.data());
            int pairs = 0, succ = 0;
            for (int i = 0; i < np; ++i) {
                pairs += v->al_kf[(size_t)i] >= 0;
                succ += v->al_succ[(size_t)i];
            }
            v->stats[6] = pairs;
            v->stats[7] = succ;
            v->poses.push_back(X);
            // stereo keyframe insertion: every kf_interval-th tracking frame,
            // when fewer than kf_permille / 1000 of the map points were good
            // at level 0, this frame's stereo points join the map (world =
            // R^T (Pc - T) with its pose) and the frame becomes a keyframe
            ++v->track_cnt;
            if (v->kf_interval > 0 && right && v->stereo_base > 0 && v->track_cnt % v->kf_interval == 0 &&
                (int)v->keyframes.size() < 8 && (double)st[0] < v->kf_permille * (double)np / 1000.0) {
                std::vector<int32_t> xs((size_t)w * h / 4 + 16), ys(xs.size()), sc(xs.size());
                const int nf = oracle_fast(cur->pyr.data(), w, h, v->p.fast_thresh, xs.data(), ys.data(), sc.data(),
                                           (int)xs.size());
                std::vector<double> pts((size_t)3 * nf + 3);
                int m = oracle_stereo_points(cur->pyr.data(), right, w, h, xs.data(), ys.data(), nf, v->max_disp,
                                             v->min_disp, v->K4, v->stereo_base, pts.data());
                const int cap = 16384 - np;  // kMaxMapPoints
                if (m > cap) m = cap;
                const double* R = cur->R;
                const double* T = cur->T;
                for (int i = 0; i < m; ++i) {
                    const double d0 = pts[(size_t)3 * i] - T[0], d1 = pts[(size_t)3 * i + 1] - T[1],
                                 d2 = pts[(size_t)3 * i + 2] - T[2];
                    for (int k = 0; k < 3; ++k)
                        v->points.push_back((R[k] * d0 + R[3 + k] * d1) + R[6 + k] * d2);
                }
                v->keyframes.push_back(cur);
                v->point_host.resize(v->points.size() / 3, (int32_t)v->keyframes.size() - 1);
                v->stats[14] = m;
                if (v->ba_iterations > 0) {
                    // photometric BA over every keyframe and the map
                    // (oracle_ba.cpp); the refined poses stay on the keyframes
                    // (the current frame's is the next frame's `last` pose)
                    const int nk = (int)v->keyframes.size();
                    std::vector<const uint8_t*> imgs((size_t)nk);
                    std::vector<double> kp((size_t)12 * nk);
                    for (int j = 0; j < nk; ++j) {
                        imgs[(size_t)j] = v->keyframes[(size_t)j]->pyr.data();
                        std::memcpy(&kp[(size_t)12 * j], v->keyframes[(size_t)j]->pose(), 12 * sizeof(double));
                    }
                    oracle_photometric_ba(imgs.data(), nk, w, h, v->K4, kp.data(), v->points.data(),
                                          v->point_host.data(), (int)(v->points.size() / 3), v->ba_iterations,
                                          nullptr);
                    for (int j = 1; j < nk; ++j) {
                        std::memcpy(v->keyframes[(size_t)j]->R, &kp[(size_t)12 * j], 9 * sizeof(double));
                        std::memcpy(v->keyframes[(size_t)j]->T, &kp[(size_t)12 * j + 9], 3 * sizeof(double));
                    }
                }
            }
            v->stats[15] = (double)v->keyframes.size();
            break;
        }
        default:
            break;
    }
    v->last_frame = cur;
    ++v->frames;
    v->stats[0] = v->state;
    v->stats[5] = v->frame_cnt;
    v->stats[11] = v->frames;
}
}  // namespace

void oracle_viso_on_new_frame(oracle_viso* v, const uint8_t* img) { on_new(v, img, nullptr); }

void oracle_viso_on_new_stereo(oracle_viso* v, const uint8_t* left, const uint8_t* right) {
    on_new(v, left, right);
}

void oracle_viso_set_bundle_adjust(oracle_viso* v, int iterations) { v->ba_iterations = iterations; }

void oracle_viso_set_keyframes(oracle_viso* v, int interval, int ngood_permille) {
    v->kf_interval = interval;
    v->kf_permille = ngood_permille;
}

void oracle_viso_set_stereo(oracle_viso* v, double baseline, int max_disp, int min_disp) {
    v->stereo_base = baseline;
    v->max_disp = max_disp;
    v->min_disp = min_disp;
}

int oracle_viso_state(const oracle_viso* v) { return v->state; }
int oracle_viso_num_poses(const oracle_viso* v) { return (int)v->poses.size(); }

void oracle_viso_poses(const oracle_viso* v, double* out12) {
    for (size_t i = 0; i < v->poses.size(); ++i) {
        quat_to_matrix(v->poses[i].q, out12 + 12 * i);
        for (int k = 0; k < 3; ++k) out12[12 * i + 9 + k] = v->poses[i].t[k];
    }
}

int oracle_viso_num_points(const oracle_viso* v) { return (int)v->points.size() / 3; }

void oracle_viso_points(const oracle_viso* v, double* out3) {
    std::memcpy(out3, v->points.data(), v->points.size() * sizeof(double));
}

void oracle_viso_last_stats(const oracle_viso* v, double* out16) {
    std::memcpy(out16, v->stats, sizeof(v->stats));
}

int oracle_viso_tracks(const oracle_viso* v, float* kp1, float* kp2, uint8_t* success, int cap) {
    int n = (int)v->kp1.size() / 2;
    int m = n < cap ? n : cap;
    if (kp1) std::memcpy(kp1, v->kp1.data(), sizeof(float) * 2 * m);
    if (kp2) std::memcpy(kp2, v->kp2.data(), sizeof(float) * 2 * m);
    if (success)
        for (int i = 0; i < m; ++i) success[i] = i < (int)v->success.size() ? v->success[(size_t)i] : 0;
    return n;
}

int oracle_viso_keyframe_poses(const oracle_viso* v, double* out12, int cap) {
    int n = (int)v->keyframes.size();
    for (int j = 0; j < n && j < cap; ++j) {
        std::memcpy(out12 + 12 * j, v->keyframes[(size_t)j]->R, 9 * sizeof(double));
        std::memcpy(out12 + 12 * j + 9, v->keyframes[(size_t)j]->T, 3 * sizeof(double));
    }
    return n;
}

int oracle_viso_alignment(const oracle_viso* v, int32_t* pair_kf, uint8_t* success,
                          double* uv_before, double* uv_after, int cap) {
    int n = (int)v->al_kf.size();
    int m = n < cap ? n : cap;
    if (pair_kf) std::memcpy(pair_kf, v->al_kf.data(), sizeof(int32_t) * m);
    if (success) std::memcpy(success, v->al_succ.data(), m);
    if (uv_before) std::memcpy(uv_before, v->al_before.data(), sizeof(double) * 2 * m);
    if (uv_after) std::memcpy(uv_after, v->al_after.data(), sizeof(double) * 2 * m);
    return n;
}

}  // extern "C"
