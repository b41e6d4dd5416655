// Exercises include/orbx_orbslam2.hpp (the ORB_SLAM2:: drop-in) through its
// reference-shaped signatures.
//   adapter_test probe                      -> prints "nodevice" if construction fails
//   adapter_test run W H img0.raw img1.raw out.bin
//        extracts both frames, matches them (window 100, 0.9, checkOri) and
//        writes: n0, kps0 (28 B each), desc0, n1, kps1, desc1, nm, matches12,
//        prev (2 floats per F1 keypoint), pyramid level 1 with its 19-px border.
//   adapter_test stereo W H left.raw right.raw mbf mb out.bin
//        extracts both images with two extractors, runs
//        OrbxFrame::ComputeStereoMatches and writes: nl, kps, desc, nr, kps,
//        desc, nkept, mvuRight, mvDepth.
//   adapter_test proj variant th ratio ori frame.bin queries.bin out.bin
//        OrbxMatcher::SearchByProjectionTable on raw tables (see test): writes
//        nmatches, q_idx, q_dist, kp_final; also runs the table twice through
//        OrbxMatcher::SearchByProjectionBatch and exits 3 if a copy differs.
//   adapter_test rgbd W H img.raw depth.raw mbf out.bin
//        extracts the image and runs OrbxFrame::ComputeStereoFromRGBD:
//        n, kps, desc, mvuRight, mvDepth.
//   adapter_test vocab voc.txt feats.raw n levelsup out.bin
//        OrbxVocabulary::loadFromTextFile + transform into std::map
//        BowVector / FeatureVector: nb, (word u32, value f64) x nb, nf,
//        (node u32, count i32, features i32 x count) x nf.
//   adapter_test aux W H rgb.raw kps.bin out.bin
//        OrbxFrameAux::ToGray (3-channel RGB image) and UndistortKeyPoints
//        (TUM1 camera) of the keypoints file (n, then n x 28 B): writes the
//        gray image (W x H) and the undistorted (x, y) pairs.
//   adapter_test time W H img.raw nfeatures reps
//        the drop-in as Frame::ExtractORB calls it (Frame.cc:259-265): prints
//        "extract_ms <median>" of ORBextractor::operator(), then
//        "pyramid_read_ms <median>" of an mvImagePyramid read after a call.
//   adapter_test time_stereo W H left.raw right.raw nfeatures mbf mb reps
//        Frame's stereo constructor: both images extracted on two threads
//        started per frame (Frame.cc:79-82), then ComputeStereoMatches through
//        OrbxFrame (Frame_orbx.cc): prints "pair_ms <median>".
//   adapter_test time_bow case.bin reps
//        OrbxMatcher::SearchByBoWTable (the SearchByBoW / SearchForTriangulation
//        forwarder, ORBmatcher_orbx.cc) on one problem from bench.py's
//        write_bow_case(): prints "bow_ms <median>" and "matches <n>".
//   adapter_test time_proj variant th ratio ori frame.bin queries.bin reps
//        OrbxMatcher::SearchByProjectionTable (the SearchByProjection / Fuse
//        forwarders, ORBmatcher_orbx.cc) on the files of "proj": prints
//        "proj_ms <median>", "proj_min_ms <min>" over reps calls and "matches <n>".
//   adapter_test time_rgbd W H img.raw depth.raw mbf reps
//        Frame's RGB-D constructor: extraction, then ComputeStereoFromRGBD
//        (Frame.cc:679-701) through OrbxFrame: prints "rgbd_frame_ms <median>"
//        and "rgbd_depth_ms <median>" (the depth call alone).
#include <algorithm>
#include <chrono>
#include <cstdio>
#include <thread>
#include <cstring>
#include <map>
#include <fstream>
#include <iostream>
#include <string>

#include "orbx_orbslam2.hpp"

using namespace ORB_SLAM2;

static cv::Mat load(const char *path, int w, int h) {
    cv::Mat m(h, w, CV_8U);
    std::ifstream f(path, std::ios::binary);
    f.read(reinterpret_cast<char *>(m.data), (std::streamsize)w * h);
    return m;
}

static void put_kps(std::ofstream &out, const std::vector<cv::KeyPoint> &ks, const cv::Mat &d) {
    const int n = (int)ks.size();
    out.write(reinterpret_cast<const char *>(&n), 4);
    for (const auto &k : ks) {
        const float f[5] = {k.pt.x, k.pt.y, k.size, k.angle, k.response};
        const int i[2] = {k.octave, k.class_id};
        out.write(reinterpret_cast<const char *>(f), 20);
        out.write(reinterpret_cast<const char *>(i), 8);
    }
    for (int r = 0; r < n; ++r) out.write(reinterpret_cast<const char *>(d.ptr<uint8_t>(r)), 32);
}

template <class F>
static double median_ms(int reps, F f) {
    std::vector<double> t(reps);
    for (int i = 0; i < reps; ++i) {
        const auto t0 = std::chrono::steady_clock::now();
        f();
        t[i] = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    }
    std::sort(t.begin(), t.end());
    return t[reps / 2];
}

int main(int argc, char **argv) {
    if (argc == 7 && std::string(argv[1]) == "time") {
        const int w = std::atoi(argv[2]), h = std::atoi(argv[3]), reps = std::atoi(argv[6]);
        cv::Mat im = load(argv[4], w, h);
        ORBextractor ex(std::atoi(argv[5]), 1.2f, 8, 20, 7);
        std::vector<cv::KeyPoint> k;
        cv::Mat d;
        for (int i = 0; i < 5; ++i) ex(im, cv::Mat(), k, d);
        std::printf("extract_ms %.4f\n", median_ms(reps, [&] { ex(im, cv::Mat(), k, d); }));
        int rows = 0;
        std::vector<double> t(reps);
        for (int i = 0; i < reps; ++i) {   // a call, then the first read of the pyramid
            ex(im, cv::Mat(), k, d);
            const auto t0 = std::chrono::steady_clock::now();
            rows += ex.mvImagePyramid[0].rows;
            t[i] = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
        }
        std::sort(t.begin(), t.end());
        std::printf("pyramid_read_ms %.4f\n", t[reps / 2]);
        std::printf("keypoints %zu rows %d\n", k.size(), rows / reps);
        return 0;
    }
    if (argc == 10 && std::string(argv[1]) == "time_stereo") {
        const int w = std::atoi(argv[2]), h = std::atoi(argv[3]), nf = std::atoi(argv[6]), reps = std::atoi(argv[9]);
        const float mbf = (float)std::atof(argv[7]), mb = (float)std::atof(argv[8]);
        cv::Mat il = load(argv[4], w, h), ir = load(argv[5], w, h);
        ORBextractor exl(nf, 1.2f, 8, 20, 7), exr(nf, 1.2f, 8, 20, 7);
        std::vector<cv::KeyPoint> kl, kr;
        cv::Mat dl, dr;
        std::vector<float> ur, dp;
        int kept = 0;
        auto pair = [&] {
            std::thread tl([&] { exl(il, cv::Mat(), kl, dl); });
            std::thread tr([&] { exr(ir, cv::Mat(), kr, dr); });
            tl.join();
            tr.join();
            kept = OrbxFrame::ComputeStereoMatches(exl, exr, kl, dl, kr, dr, mbf, mb, ur, dp);
        };
        for (int i = 0; i < 5; ++i) pair();
        std::printf("pair_ms %.4f\n", median_ms(reps, pair));
        std::printf("keypoints %zu %zu kept %d\n", kl.size(), kr.size(), kept);
        return 0;
    }
    if (argc == 4 && std::string(argv[1]) == "time_bow") {
        std::ifstream f(argv[2], std::ios::binary);
        auto rd = [&](void *p, size_t n) { f.read(reinterpret_cast<char *>(p), (std::streamsize)n); };
        int32_t hd[5];   // variant, nlevels, checkOri, ntri, (pad)
        float nnratio;
        rd(hd, sizeof(hd));
        rd(&nnratio, 4);
        std::vector<float> tri(hd[3]);
        rd(tri.data(), 4 * tri.size());
        struct Side { std::vector<orbx_keypoint> k; std::vector<uint8_t> d, fl; std::vector<uint32_t> ids;
                      std::vector<int32_t> off, feat; orbx_bow_side s; } S[2];
        for (Side &x : S) {
            int32_t n, nn, nf;
            rd(&n, 4); rd(&nn, 4); rd(&nf, 4);
            x.k.resize(n); x.d.resize(32 * (size_t)n); x.fl.resize(n); x.ids.resize(nn); x.off.resize(nn + 1);
            x.feat.resize(std::max(nf, 1));
            rd(x.k.data(), sizeof(orbx_keypoint) * n); rd(x.d.data(), x.d.size()); rd(x.fl.data(), n);
            rd(x.ids.data(), 4 * (size_t)nn); rd(x.off.data(), 4 * (size_t)(nn + 1)); rd(x.feat.data(), 4 * (size_t)nf);
            x.s = orbx_bow_side{x.k.data(), x.d.data(), x.fl.data(), n, x.ids.data(), x.off.data(), x.feat.data(), nn};
        }
        if (!f) { std::fprintf(stderr, "short case file\n"); return 2; }
        const int reps = std::atoi(argv[3]);
        std::vector<int> ma, mb;
        int nm = 0;
        auto call = [&] { nm = OrbxMatcher::SearchByBoWTable(hd[0], S[0].s, S[1].s, nnratio, hd[2] != 0, tri, hd[1], ma, mb); };
        for (int i = 0; i < 5; ++i) call();
        std::printf("bow_ms %.4f\n", median_ms(reps, call));
        std::printf("matches %d\n", nm);
        return 0;
    }
    if (argc == 8 && std::string(argv[1]) == "time_rgbd") {
        const int w = std::atoi(argv[2]), h = std::atoi(argv[3]), reps = std::atoi(argv[7]);
        const float mbf = (float)std::atof(argv[6]);
        cv::Mat im = load(argv[4], w, h);
        cv::Mat dm(h, w, CV_32F);
        {
            std::ifstream f(argv[5], std::ios::binary);
            f.read(reinterpret_cast<char *>(dm.data), (std::streamsize)w * h * 4);
        }
        ORBextractor ex(1000, 1.2f, 8, 20, 7);
        std::vector<cv::KeyPoint> k;
        cv::Mat d;
        std::vector<float> ur, dp;
        auto depth = [&] { OrbxFrame::ComputeStereoFromRGBD(k, k, dm, mbf, ur, dp); };
        auto frame = [&] { ex(im, cv::Mat(), k, d); depth(); };
        for (int i = 0; i < 5; ++i) frame();
        std::printf("rgbd_frame_ms %.4f\n", median_ms(reps, frame));
        std::printf("rgbd_depth_ms %.4f\n", median_ms(reps, depth));
        int nd = 0;
        for (float v : dp) nd += v > 0;
        std::printf("keypoints %zu depths %d\n", k.size(), nd);
        return 0;
    }
    if (argc >= 2 && std::string(argv[1]) == "probe") {
        try {
            ORBextractor ex(1000, 1.2f, 8, 20, 7);
            std::cout << "levels " << ex.GetLevels() << " scale " << ex.GetScaleFactor() << "\n";
        } catch (const std::runtime_error &e) {
            std::cout << "nodevice\n";
        }
        return 0;
    }
    if (argc == 9 && std::string(argv[1]) == "stereo") {
        const int w = std::atoi(argv[2]), h = std::atoi(argv[3]);
        cv::Mat il = load(argv[4], w, h), ir = load(argv[5], w, h);
        ORBextractor exl(1000, 1.2f, 8, 20, 7), exr(1000, 1.2f, 8, 20, 7);
        std::vector<cv::KeyPoint> kl, kr;
        cv::Mat dl, dr;
        exl(il, cv::Mat(), kl, dl);
        exr(ir, cv::Mat(), kr, dr);
        std::vector<float> ur, dp;
        const int kept = OrbxFrame::ComputeStereoMatches(exl, exr, kl, dl, kr, dr, (float)std::atof(argv[6]),
                                                         (float)std::atof(argv[7]), ur, dp);
        std::ofstream out(argv[8], std::ios::binary);
        put_kps(out, kl, dl);
        put_kps(out, kr, dr);
        out.write(reinterpret_cast<const char *>(&kept), 4);
        out.write(reinterpret_cast<const char *>(ur.data()), 4 * ur.size());
        out.write(reinterpret_cast<const char *>(dp.data()), 4 * dp.size());
        return 0;
    }
    if ((argc == 9 && std::string(argv[1]) == "proj") || (argc == 9 && std::string(argv[1]) == "time_proj")) {
        // frame.bin: n, min_x, max_x, min_y, max_y, n x 28 B keys, n x 32 B desc, n floats uright, n u8 state,
        //            nlev, nlev floats inv_sigma2;  queries.bin: nq, nq x 36 B rows, nq x 32 B desc
        std::ifstream ff(argv[6], std::ios::binary), fq(argv[7], std::ios::binary);
        int n = 0, nq = 0, nlev = 0;
        float b[4];
        ff.read(reinterpret_cast<char *>(&n), 4);
        ff.read(reinterpret_cast<char *>(b), 16);
        std::vector<orbx_keypoint> kr(n);
        ff.read(reinterpret_cast<char *>(kr.data()), 28 * (std::streamsize)n);
        std::vector<cv::KeyPoint> keys;
        for (const auto &k : kr)
            keys.push_back(cv::KeyPoint(cv::Point2f(k.x, k.y), k.size, k.angle, k.response, k.octave, k.class_id));
        cv::Mat desc(n, 32, CV_8U);
        ff.read(reinterpret_cast<char *>(desc.data), 32 * (std::streamsize)n);
        std::vector<float> ur(n);
        ff.read(reinterpret_cast<char *>(ur.data()), 4 * (std::streamsize)n);
        std::vector<uint8_t> st(n);
        ff.read(reinterpret_cast<char *>(st.data()), n);
        ff.read(reinterpret_cast<char *>(&nlev), 4);
        std::vector<float> isg(nlev);
        ff.read(reinterpret_cast<char *>(isg.data()), 4 * (std::streamsize)nlev);
        fq.read(reinterpret_cast<char *>(&nq), 4);
        std::vector<orbx_proj_query> q(nq);
        fq.read(reinterpret_cast<char *>(q.data()), sizeof(orbx_proj_query) * (std::streamsize)nq);
        cv::Mat qd(nq, 32, CV_8U);
        fq.read(reinterpret_cast<char *>(qd.data), 32 * (std::streamsize)nq);
        OrbxMatcher::ProjFrame F;
        F.keys = &keys; F.desc = &desc; F.uright = &ur; F.mp_state = &st; F.inv_sigma2 = &isg;
        F.min_x = b[0]; F.max_x = b[1]; F.min_y = b[2]; F.max_y = b[3];
        std::vector<int> qi, qdist, kf;
        const int nm = OrbxMatcher::SearchByProjectionTable(std::atoi(argv[2]), F, q, qd, std::atoi(argv[3]),
                                                            (float)std::atof(argv[4]), std::atoi(argv[5]) != 0, qi,
                                                            qdist, kf);
        if (std::string(argv[1]) == "time_proj") {
            const int reps = std::max(1, std::atoi(argv[8]));
            std::vector<double> t(reps);
            for (int i = 0; i < reps; ++i) {
                const auto t0 = std::chrono::steady_clock::now();
                OrbxMatcher::SearchByProjectionTable(std::atoi(argv[2]), F, q, qd, std::atoi(argv[3]),
                                                     (float)std::atof(argv[4]), std::atoi(argv[5]) != 0, qi, qdist, kf);
                t[i] = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
            }
            std::sort(t.begin(), t.end());
            std::printf("proj_ms %.4f\nproj_min_ms %.4f\nmatches %d\n", t[reps / 2], t[0], nm);
            return 0;
        }
        // the same problem twice through the batch entry point: both copies
        // must equal the single call (a non-zero exit says they do not)
        std::vector<std::vector<int>> bqi, bqd, bkf;
        const std::vector<int> bnm = OrbxMatcher::SearchByProjectionBatch(
            std::atoi(argv[2]), {F, F}, {q, q}, {qd, qd}, std::atoi(argv[3]), (float)std::atof(argv[4]),
            std::atoi(argv[5]) != 0, bqi, bqd, bkf);
        for (int i = 0; i < 2; ++i)
            if (bnm[i] != nm || bqi[i] != qi || bqd[i] != qdist || bkf[i] != kf) {
                std::cerr << "batch problem " << i << " differs from the single call\n";
                return 3;
            }
        std::ofstream out(argv[8], std::ios::binary);
        out.write(reinterpret_cast<const char *>(&nm), 4);
        out.write(reinterpret_cast<const char *>(qi.data()), 4 * qi.size());
        out.write(reinterpret_cast<const char *>(qdist.data()), 4 * qdist.size());
        out.write(reinterpret_cast<const char *>(kf.data()), 4 * kf.size());
        return 0;
    }
    if (argc == 8 && std::string(argv[1]) == "rgbd") {
        const int w = std::atoi(argv[2]), h = std::atoi(argv[3]);
        cv::Mat im = load(argv[4], w, h);
        cv::Mat depth(h, w, CV_32F);
        std::ifstream f(argv[5], std::ios::binary);
        f.read(reinterpret_cast<char *>(depth.data), (std::streamsize)4 * w * h);
        ORBextractor ex(1000, 1.2f, 8, 20, 7);
        std::vector<cv::KeyPoint> k;
        cv::Mat d;
        ex(im, cv::Mat(), k, d);
        std::vector<float> ur, dp;
        OrbxFrame::ComputeStereoFromRGBD(k, k, depth, (float)std::atof(argv[6]), ur, dp);
        std::ofstream out(argv[7], std::ios::binary);
        put_kps(out, k, d);
        out.write(reinterpret_cast<const char *>(ur.data()), 4 * ur.size());
        out.write(reinterpret_cast<const char *>(dp.data()), 4 * dp.size());
        return 0;
    }
    if (argc == 7 && std::string(argv[1]) == "vocab") {
        OrbxVocabulary voc;
        if (!voc.loadFromTextFile(argv[2])) return 3;
        const int n = std::atoi(argv[4]), levelsup = std::atoi(argv[5]);
        std::ifstream f(argv[3], std::ios::binary);
        std::vector<cv::Mat> feats;
        for (int i = 0; i < n; ++i) {
            cv::Mat d(1, 32, CV_8U);
            f.read(reinterpret_cast<char *>(d.data), 32);
            feats.push_back(d);
        }
        std::map<unsigned int, double> bow;
        std::map<unsigned int, std::vector<unsigned int>> fv;
        voc.transform(feats, bow, fv, levelsup);
        std::ofstream out(argv[6], std::ios::binary);
        const int nb = (int)bow.size(), nf = (int)fv.size();
        out.write(reinterpret_cast<const char *>(&nb), 4);
        for (const auto &kv : bow) {
            out.write(reinterpret_cast<const char *>(&kv.first), 4);
            out.write(reinterpret_cast<const char *>(&kv.second), 8);
        }
        out.write(reinterpret_cast<const char *>(&nf), 4);
        for (const auto &kv : fv) {
            const int c = (int)kv.second.size();
            out.write(reinterpret_cast<const char *>(&kv.first), 4);
            out.write(reinterpret_cast<const char *>(&c), 4);
            out.write(reinterpret_cast<const char *>(kv.second.data()), 4 * (std::streamsize)c);
        }
        return 0;
    }
    if (argc == 7 && std::string(argv[1]) == "aux") {
        const int w = std::atoi(argv[2]), h = std::atoi(argv[3]);
        cv::Mat im(h, w, CV_8UC3);
        std::ifstream fi(argv[4], std::ios::binary);
        fi.read(reinterpret_cast<char *>(im.data), (std::streamsize)w * h * 3);
        OrbxFrameAux::ToGray(im, true);
        std::ifstream fk(argv[5], std::ios::binary);
        int n = 0;
        fk.read(reinterpret_cast<char *>(&n), 4);
        std::vector<cv::KeyPoint> kps(n);
        for (auto &k : kps) {
            float f[5];
            int i[2];
            fk.read(reinterpret_cast<char *>(f), 20);
            fk.read(reinterpret_cast<char *>(i), 8);
            k = cv::KeyPoint(cv::Point2f(f[0], f[1]), f[2], f[3], f[4], i[0], i[1]);
        }
        cv::Mat K(3, 3, CV_32F), D(5, 1, CV_32F);
        const float kv[9] = {517.306408f, 0, 318.643040f, 0, 516.469215f, 255.313989f, 0, 0, 1};
        const float dv[5] = {0.262383f, -0.953104f, -0.005358f, 0.002628f, 1.163314f};
        std::memcpy(K.data, kv, sizeof(kv));
        std::memcpy(D.data, dv, sizeof(dv));
        std::vector<cv::KeyPoint> un;
        OrbxFrameAux::UndistortKeyPoints(kps, K, D, un);
        std::ofstream out(argv[6], std::ios::binary);
        out.write(reinterpret_cast<const char *>(im.data), (std::streamsize)w * h);
        for (const auto &k : un) {
            out.write(reinterpret_cast<const char *>(&k.pt.x), 4);
            out.write(reinterpret_cast<const char *>(&k.pt.y), 4);
        }
        return 0;
    }
    if (argc != 7 || std::string(argv[1]) != "run") return 2;
    const int w = std::atoi(argv[2]), h = std::atoi(argv[3]);
    cv::Mat im0 = load(argv[4], w, h), im1 = load(argv[5], w, h);
    ORBextractor ex(1000, 1.2f, 8, 20, 7);
    std::vector<cv::KeyPoint> k0, k1;
    cv::Mat d0, d1;
    ex(im0, cv::Mat(), k0, d0);
    ex(im1, cv::Mat(), k1, d1);
    std::vector<cv::Point2f> prev(k0.size());
    for (size_t i = 0; i < k0.size(); ++i) prev[i] = k0[i].pt;
    std::vector<int> m12;
    const int nm = OrbxMatcher::SearchForInitialization(k0, d0, k1, d1, w, h, prev, m12, 100, 0.9f, true);
    std::ofstream out(argv[6], std::ios::binary);
    put_kps(out, k0, d0);
    put_kps(out, k1, d1);
    out.write(reinterpret_cast<const char *>(&nm), 4);
    out.write(reinterpret_cast<const char *>(m12.data()), 4 * m12.size());
    for (const auto &p : prev) { out.write(reinterpret_cast<const char *>(&p.x), 4); out.write(reinterpret_cast<const char *>(&p.y), 4); }
    const cv::Mat &l1 = ex.mvImagePyramid[1];
    const int bw = l1.cols + 38, bh = l1.rows + 38;
    out.write(reinterpret_cast<const char *>(&bw), 4);
    out.write(reinterpret_cast<const char *>(&bh), 4);
    const uint8_t *base = l1.data - 19 * l1.step - 19;
    for (int y = 0; y < bh; ++y) out.write(reinterpret_cast<const char *>(base + y * l1.step), bw);
    return 0;
}
