// stereo_matching.hpp — header-only C++ facade with the reference's class API over sm_capi.h.
//
// Source-compatible with the reference driver's use of class StereoMatching (main_.cpp:130-178):
// a user replaces `#include "stereoMatching.h"` and OpenCV's Mat/imread/pyrDown by this header
// (`using namespace smamd;` in place of `using namespace cv;`) and keeps the call sequence:
//
//   string StereoMatching::costcalculation = "censusGrad";     // main_.cpp:15-19: the program
//   string StereoMatching::aggregation = "CBCA";               // defines the static selectors,
//   string StereoMatching::optimization = "sgm";               // exactly as the reference's
//   string StereoMatching::object = "";                        // header declares them (h:50-54)
//   const string StereoMatching::root = "...";
//   ...
//   StereoMatching::Parameters param(maxDisp, rows, cols, lamCen, lamG, M, lamc, ts, csv, disSc);  // main:138
//   smPsy[p] = new StereoMatching(I1_c, I2_c, I1, I2, DT, all, nonocc, disc, param);              // main:139
//   smPsy[p]->costCalculate();                                  // cpp:945-1021
//   pyrDown(I1_c, I1_c); ...                                    // main:145-154
//   SolveAll(smPsy, PY_LEV, REG_LAMBDA);                        // cpp:2142-2208
//   smPsy[0]->openCSV(); smPsy[0]->dispOptimize();              // main:159-163, cpp:1046-1136
//   if (StereoMatching::Do_refine) smPsy[0]->refine();          // main:165-166
//   smPsy[0]->closeCSV(); smPsy[0]->saveTime(time, "all");      // main:168-171
//   const int16_t* d = smPsy[0]->DP[0].ptr<int16_t>(0);         // public member DP (h:2724)
//
// smamd::Mat mirrors the part of cv::Mat the driver touches: reference-counted shallow copies
// (the reference's ctor keeps headers of the caller's images, cpp:2066-2075), rows/cols/step/data,
// empty(), channels(), ptr<T>(row), convertTo(CV_32F, alpha).  imread reads PNG (main_.cpp:92-107
// reads the Middlebury *.png files; decoded here with zlib, link -lz) and binary PNM (P5 gray, P6
// colour): flags 1 -> 3-channel BGR, 0 -> gray with libpng's rgb_to_gray weights, the formula
// OpenCV's PNG decoder uses.  All compute runs in libsm_hip.so on
// the GPU; the library does no file I/O, so openCSV/closeCSV/saveTime keep their records in memory
// (the reference wrote savePath files and exit()ed on failure, h:1727-1744).  Non-OK statuses
// become std::runtime_error (the reference threw cv::Exception from CV_Assert).
#pragma once
#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <ctime>
#include <fstream>
#include <iostream>
#include <iterator>
#include <memory>
#include <new>
#include <sstream>
#include <stdexcept>
#include <string>
#include <vector>

#include "sm_capi.h"

#if __has_include(<zlib.h>)
#include <zlib.h>
#define SMAMD_HAVE_PNG 1
#else
#define SMAMD_HAVE_PNG 0
#endif

namespace smamd {

// OpenCV depth codes used by the driver (CV_8U images, CV_16S DP, CV_32F DT)
enum { CV_8U = 0, CV_16S = 3, CV_32F = 5 };

#ifndef CV_Assert
#define CV_Assert(expr) \
    do { if (!(expr)) throw std::runtime_error("Assertion failed: " #expr); } while (0)
#endif

inline int& default_device() {   // HIP device for the free functions (pyrDown); ctor takes its own
    static int dev = 0;
    return dev;
}

class Mat {
   public:
    int rows = 0, cols = 0;
    size_t step = 0;             // bytes per row
    uint8_t* data = nullptr;

    Mat() = default;
    Mat(int nrows, int ncols, int depth, int channels = 1) { create(nrows, ncols, depth, channels); }
    // non-owning view of caller memory (e.g. a cv::Mat: view(m.rows, m.cols, m.channels(), m.step, m.data))
    static Mat view(int nrows, int ncols, int channels, size_t row_step, const void* ptr0, int depth = CV_8U) {
        Mat m;
        m.rows = nrows, m.cols = ncols, m.cn_ = channels, m.depth_ = depth, m.step = row_step;
        m.data = (uint8_t*)ptr0;
        return m;
    }
    void create(int nrows, int ncols, int depth, int channels = 1) {
        rows = nrows, cols = ncols, depth_ = depth, cn_ = channels;
        step = (size_t)cols * elemSize();
        buf_ = std::make_shared<std::vector<uint8_t>>(step * rows);
        data = buf_->data();
    }
    bool empty() const { return data == nullptr || rows == 0 || cols == 0; }
    int channels() const { return cn_; }
    int depth() const { return depth_; }
    int type() const { return depth_ + ((cn_ - 1) << 3); }   // CV_MAKETYPE
    size_t elemSize1() const { return depth_ == CV_8U ? 1 : depth_ == CV_16S ? 2 : 4; }
    size_t elemSize() const { return elemSize1() * cn_; }
    bool isContinuous() const { return step == (size_t)cols * elemSize(); }
    template <typename T> T* ptr(int r = 0) { return (T*)(data + (size_t)r * step); }
    template <typename T> const T* ptr(int r = 0) const { return (const T*)(data + (size_t)r * step); }
    Mat clone() const {
        Mat m(rows, cols, depth_, cn_);
        for (int r = 0; r < rows; r++) std::memcpy(m.ptr<uint8_t>(r), ptr<uint8_t>(r), (size_t)cols * elemSize());
        return m;
    }
    // Mat::convertTo(dst, rtype, alpha, beta) for u8 / s16 / f32 -> f32 (main_.cpp:127-129:
    // DT.convertTo(DT, CV_32F, 1.0 / disp_reduceCoeff)): (float)v * (float)alpha + (float)beta
    void convertTo(Mat& dst, int rtype, double alpha = 1, double beta = 0) const {
        if (rtype != CV_32F) throw std::invalid_argument("convertTo: only CV_32F targets are supported");
        Mat out(rows, cols, CV_32F, cn_);
        const float a = (float)alpha, b = (float)beta;
        for (int r = 0; r < rows; r++) {
            float* o = out.ptr<float>(r);
            for (int i = 0; i < cols * cn_; i++) {
                const float v = depth_ == CV_8U ? (float)ptr<uint8_t>(r)[i]
                                : depth_ == CV_16S ? (float)ptr<int16_t>(r)[i] : ptr<float>(r)[i];
                o[i] = b == 0.f ? v * a : v * a + b;
            }
        }
        dst = out;   // a new buffer; other headers of the old one keep it (cv::Mat semantics)
    }
    // rows x cols x channels packed copy of the pixels (host), element type T
    template <typename T> std::vector<T> packed() const {
        std::vector<T> v((size_t)rows * cols * cn_);
        for (int r = 0; r < rows; r++) std::memcpy(v.data() + (size_t)r * cols * cn_, ptr<uint8_t>(r), (size_t)cols * elemSize());
        return v;
    }

   private:
    int depth_ = CV_8U, cn_ = 1;
    std::shared_ptr<std::vector<uint8_t>> buf_;
};

namespace detail {

// Largest image imread accepts (pixels): header sizes above it, or whose products would overflow,
// are rejected before anything is allocated (a crafted header must not wrap a buffer size).
constexpr uint64_t kMaxImagePixels = 1ull << 28;
inline bool size_ok(int64_t w, int64_t h) { return w >= 1 && h >= 1 && (uint64_t)w * (uint64_t)h <= kMaxImagePixels; }

// Decoded 8-bit pixels: w x h, cin = 1 (gray) or 3 (R, G, B), row-major.
struct Pixels {
    int w = 0, h = 0, cin = 0;
    std::vector<uint8_t> px;
};

inline bool read_pnm(std::ifstream& f, Pixels& out) {
    std::string magic;
    int w = 0, h = 0, maxv = 0;
    if (!(f >> magic >> w >> h >> maxv) || (magic != "P6" && magic != "P5") || maxv != 255 || !size_ok(w, h))
        return false;
    f.get();
    out.w = w, out.h = h, out.cin = magic == "P6" ? 3 : 1;
    out.px.resize((size_t)w * h * out.cin);
    return (bool)f.read((char*)out.px.data(), (std::streamsize)out.px.size());
}

#if SMAMD_HAVE_PNG
inline uint32_t be32(const uint8_t* p) { return (uint32_t)p[0] << 24 | (uint32_t)p[1] << 16 | (uint32_t)p[2] << 8 | p[3]; }

// PNG (ISO/IEC 15948) the way OpenCV's PngDecoder delivers it to imread(.., 0 / 1): 8-bit samples
// (1/2/4-bit gray expanded to 8 bits, 16-bit samples stripped to their high byte as
// png_set_strip_16 does, palettes expanded to RGB, alpha dropped).  Non-interlaced images only.
inline bool read_png(const std::vector<uint8_t>& file, Pixels& out) {
    static const uint8_t sig[8] = {0x89, 'P', 'N', 'G', 0x0d, 0x0a, 0x1a, 0x0a};
    if (file.size() < 8 || std::memcmp(file.data(), sig, 8) != 0) return false;
    int64_t w = 0, h = 0;
    int depth = 0, ctype = -1, interlace = 0;
    std::vector<uint8_t> idat, plte;
    for (size_t pos = 8; pos + 12 <= file.size();) {
        const uint32_t len = be32(&file[pos]);
        if (pos + 12 + (size_t)len > file.size()) return false;
        const uint8_t* type = &file[pos + 4];
        const uint8_t* data = &file[pos + 8];
        if (!std::memcmp(type, "IHDR", 4) && len >= 13) {
            w = be32(data), h = be32(data + 4), depth = data[8], ctype = data[9], interlace = data[12];
        } else if (!std::memcmp(type, "PLTE", 4)) {
            plte.assign(data, data + len);
        } else if (!std::memcmp(type, "IDAT", 4)) {
            idat.insert(idat.end(), data, data + len);
        } else if (!std::memcmp(type, "IEND", 4)) {
            break;
        }
        pos += 12 + (size_t)len;
    }
    // samples per pixel by colour type: 0 gray, 2 RGB, 3 palette index, 4 gray + alpha, 6 RGBA
    const int spp = ctype == 0 ? 1 : ctype == 2 ? 3 : ctype == 3 ? 1 : ctype == 4 ? 2 : ctype == 6 ? 4 : 0;
    const bool depth_ok = depth == 8 || depth == 16 || ((ctype == 0 || ctype == 3) && (depth == 1 || depth == 2 || depth == 4));
    // (w * h <= 2^28 keeps every size below in 64-bit range: stride <= 8 w + 1)
    if (!size_ok(w, h) || spp == 0 || !depth_ok || interlace != 0 || (ctype == 3 && (plte.empty() || depth == 16)))
        return false;
    const size_t bpp = std::max<size_t>(1, (size_t)spp * depth / 8);     // filter byte distance
    const size_t stride = ((size_t)w * spp * depth + 7) / 8;             // bytes per scanline
    // zlib's deflate expands at most ~1032:1: an IDAT far too short for the header's size is
    // rejected before the scanline buffer is allocated
    if ((uint64_t)h * (stride + 1) > (uint64_t)idat.size() * 1100 + 4096) return false;
    std::vector<uint8_t> raw(h * (stride + 1));
    uLongf rlen = (uLongf)raw.size();
    if (uncompress(raw.data(), &rlen, idat.data(), (uLong)idat.size()) != Z_OK || rlen != raw.size()) return false;
    // undo the per-scanline filters (None, Sub, Up, Average, Paeth)
    std::vector<uint8_t> img((size_t)h * stride);
    for (int y = 0; y < h; y++) {
        const uint8_t ft = raw[(size_t)y * (stride + 1)];
        const uint8_t* src = &raw[(size_t)y * (stride + 1) + 1];
        uint8_t* cur = &img[(size_t)y * stride];
        const uint8_t* up = y > 0 ? &img[(size_t)(y - 1) * stride] : nullptr;
        for (size_t i = 0; i < stride; i++) {
            const int a = i >= bpp ? cur[i - bpp] : 0, b = up ? up[i] : 0, c = (up && i >= bpp) ? up[i - bpp] : 0;
            int x = src[i];
            switch (ft) {
                case 0: break;
                case 1: x += a; break;
                case 2: x += b; break;
                case 3: x += (a + b) / 2; break;
                case 4: {
                    const int p = a + b - c, pa = std::abs(p - a), pb = std::abs(p - b), pc = std::abs(p - c);
                    x += (pa <= pb && pa <= pc) ? a : (pb <= pc ? b : c);
                    break;
                }
                default: return false;
            }
            cur[i] = (uint8_t)x;
        }
    }
    out.w = (int)w, out.h = (int)h, out.cin = (ctype == 0 || ctype == 4) ? 1 : 3;
    out.px.assign((size_t)w * h * out.cin, 0);
    for (int y = 0; y < h; y++) {
        const uint8_t* row = &img[(size_t)y * stride];
        for (int x = 0; x < w; x++) {
            uint8_t* o = &out.px[((size_t)y * w + x) * out.cin];
            if (depth < 8) {   // packed gray / palette indices, most significant bits first
                const int per = 8 / depth, shift = 8 - depth * (x % per + 1);
                const int v = (row[x / per] >> shift) & ((1 << depth) - 1);
                if (ctype == 3) {
                    if ((size_t)v * 3 + 2 >= plte.size()) return false;
                    o[0] = plte[v * 3], o[1] = plte[v * 3 + 1], o[2] = plte[v * 3 + 2];
                } else {
                    o[0] = (uint8_t)(v * 255 / ((1 << depth) - 1));
                }
                continue;
            }
            const size_t bs = depth / 8;   // bytes per sample; 16-bit: the high byte comes first
            const uint8_t* p = row + (size_t)x * spp * bs;
            if (ctype == 3) {
                const int v = p[0];
                if ((size_t)v * 3 + 2 >= plte.size()) return false;
                o[0] = plte[v * 3], o[1] = plte[v * 3 + 1], o[2] = plte[v * 3 + 2];
            } else {
                for (int k = 0; k < out.cin; k++) o[k] = p[k * bs];
            }
        }
    }
    return true;
}
#endif

inline Mat imread_impl(const std::string& path, int flags) {
    std::ifstream f(path, std::ios::binary);
    if (!f) return Mat();
    detail::Pixels d;
    const int first = f.peek();
#if SMAMD_HAVE_PNG
    if (first == 0x89) {
        std::vector<uint8_t> file((std::istreambuf_iterator<char>(f)), std::istreambuf_iterator<char>());
        if (!detail::read_png(file, d)) return Mat();
    } else
#endif
        if (first != 'P' || !detail::read_pnm(f, d)) {
        return Mat();
    }
    const int w = d.w, h = d.h, cin = d.cin;
    const std::vector<uint8_t>& px = d.px;
    Mat m(h, w, CV_8U, flags == 0 ? 1 : 3);
    for (size_t i = 0; i < (size_t)w * h; i++) {
        const uint8_t R = px[i * cin], G = px[i * cin + (cin - 1) / 2], B = px[i * cin + cin - 1];
        if (flags == 0) {
            m.data[i] = cin == 1 ? R : (uint8_t)((R * 9798 + G * 19235 + B * 3735 + 16384) >> 15);
        } else {
            m.data[i * 3] = B, m.data[i * 3 + 1] = G, m.data[i * 3 + 2] = R;
        }
    }
    return m;
}
}  // namespace detail

// cv::imread for PNG (when zlib is available) and binary PNM (P6 RGB / P5 gray, maxval 255).
// flags 1: 3-channel BGR; flags 0: gray ((R*9798 + G*19235 + B*3735 + 16384) >> 15, libpng's
// rgb_to_gray).  Empty Mat on failure (main_.cpp:108 tests empty()).
inline Mat imread(const std::string& path, int flags = 1) {
    try {
        return detail::imread_impl(path, flags);
    } catch (const std::bad_alloc&) {   // an image too large for this host: empty Mat, as documented
        return Mat();
    } catch (const std::length_error&) {
        return Mat();
    }
}

// cv::pyrDown (main_.cpp:145-154) on the GPU: u8 with 1 or 3 channels (the inputs, masks) or
// 1-channel f32 (the ground truth DT).  dst gets a new buffer of (rows+1)/2 x (cols+1)/2.
inline void pyrDown(const Mat& src, Mat& dst) {
    if (src.empty()) throw std::invalid_argument("pyrDown: empty source");
    Mat out((src.rows + 1) / 2, (src.cols + 1) / 2, src.depth(), src.channels());
    sm_status s;
    if (src.depth() == CV_8U) {
        const std::vector<uint8_t> in = src.packed<uint8_t>();
        s = sm_pyr_down(default_device(), in.data(), src.rows, src.cols, src.channels(), out.data);
    } else if (src.depth() == CV_32F && src.channels() == 1) {
        const std::vector<float> in = src.packed<float>();
        s = sm_pyr_down_f32(default_device(), in.data(), src.rows, src.cols, (float*)out.data);
    } else {
        throw std::invalid_argument("pyrDown: u8 (1/3 channels) or 1-channel f32 only");
    }
    if (s != SM_OK) throw std::runtime_error(std::string("pyrDown: ") + sm_status_string(s));
    dst = out;
}

class StereoMatching {
   public:
    // static selectors (h:50-54): declared here, defined once by the program (main_.cpp:15-19)
    static const std::string root;
    static std::string costcalculation;
    static std::string aggregation;
    static std::string optimization;
    static std::string object;
    // compile-time switches (h:57-83); static const in the reference, settable here before a ctor
    static constexpr bool preMedBlur = false;      // h:66
    inline static bool Do_refine = false;          // h:70
    static constexpr bool Do_LRConsis = true;      // h:72
    inline static bool Do_regionVote = true;       // h:75
    inline static bool Do_properIpol = true;       // h:76
    inline static bool Do_lastMedianBlur = true;   // h:80
    // `#define MY_GUIDE` (h:38, commented out in the shipped build) as a switch: false = GF runs
    // cv::ximgproc::guidedFilter (cpp:4513), true = guideFilterCore_matlab (cpp:4509)
    inline static bool gf_my_guide = false;

    struct Parameters {  // StereoMatching::Parameters (h:85-351), the fields the hot path reads
        int numDisparities, rows, cols;
        int lamCen, lamG, disSc;
        int vmTop_Num, ts;
        float vmTop_thres;
        std::string errCsvName;
        int censusFunc = 3;                   // h:244
        int cbca_iterationNum = 2, cbca_minArmL = 1;
        int cbca_crossL0 = 17, cbca_crossL_out0 = 34, cbca_cTresh0 = 20, cbca_cTresh_out0 = 6;
        int sgm_scanNum = 4, sgm_corDifThres = 15, sgm_reduCoeffi1 = 4;
        int errorThreshold = 1;               // h:225
        float LRmaxDiff = 0;                  // h:212
        int DISP_OCC = -2 * 16;               // h:216
        int region_vote_nums = 2;             // h:306
        // Parameters(maxDisp, h, w, lamCen, lamG, M, lamc, ts, errCsvName, disSc) — main_.cpp:138
        Parameters(int maxDisp, int h, int w, int lamCen_ = 13, int lamG_ = 1, int M = 2, int lamc = 109,
                   int ts_ = 10, const std::string& errCsvName_ = "", int disSc_ = 1)
            : numDisparities(maxDisp + 1), rows(h), cols(w), lamCen(lamCen_), lamG(lamG_), disSc(disSc_),
              vmTop_Num(M), ts(ts_), vmTop_thres(lamc * 0.01f), errCsvName(errCsvName_) {}
    };

    struct RegionErr {            // one line of calErr's report (h:1798-1799)
        std::string region;
        float PBM, RMS;
    };

    // StereoMatching(I1_c, I2_c, I1_g, I2_g, DT, all_mask, nonocc_mask, disc_mask, param) — cpp:2058;
    // main_.cpp:139.  DT and the masks are kept (shallow, like the reference's headers) for calErr.
    StereoMatching(Mat& I1_c, Mat& I2_c, Mat& I1_g, Mat& I2_g, Mat& DT_, Mat& all_mask, Mat& nonocc_mask,
                   Mat& disc_mask, const Parameters& param, int hip_device = 0)
        : param_(param), h_(I1_c.rows), w_(I1_c.cols), d_(param.numDisparities) {
        DT = DT_;
        I_mask[0] = nonocc_mask;   // cpp:2073-2075
        I_mask[1] = all_mask;
        I_mask[2] = disc_mask;
        init_or_release(I1_c, I2_c, I1_g, I2_g, hip_device);
    }
    // without ground truth (no calErr)
    StereoMatching(const Mat& I1_c, const Mat& I2_c, const Mat& I1_g, const Mat& I2_g, const Parameters& param,
                   int hip_device = 0)
        : param_(param), h_(I1_c.rows), w_(I1_c.cols), d_(param.numDisparities) {
        init_or_release(I1_c, I2_c, I1_g, I2_g, hip_device);
    }
    ~StereoMatching() { sm_destroy(ctx_); }
    StereoMatching(const StereoMatching&) = delete;
    StereoMatching& operator=(const StereoMatching&) = delete;

    void costCalculate() { check(sm_cost_calculate(ctx_), "costCalculate"); }
    void dispOptimize() {  // DP[0] (and DP[1] when Do_refine, or with "so": cpp:1093), cpp:1046-1136
        DP[0].create(h_, w_, CV_16S);
        check(sm_disp_optimize(ctx_, DP[0].ptr<int16_t>()), "dispOptimize");
        if (refine_on_ || (optimization == "so" && Do_LRConsis)) {
            DP[1].create(h_, w_, CV_16S);
            check(sm_get_disp(ctx_, 1, DP[1].ptr<int16_t>()), "DP[1]");
        }
    }
    void refine() {  // cpp:1138-1511; needs Do_refine at construction
        DP[0].create(h_, w_, CV_16S);
        check(sm_refine(ctx_, DP[0].ptr<int16_t>()), "refine");
    }
    void pipeline() {  // cpp:1950-1981 (no SolveAll)
        costCalculate();
        dispOptimize();
        if (Do_refine) refine();
    }
    std::vector<float> volume(int view = 0) {   // public member vm[view] (h:2720)
        std::vector<float> v((size_t)h_ * w_ * d_);
        check(sm_get_volume(ctx_, view, v.data()), "vm");
        return v;
    }

    // CSV of per-object error ratios (cpp:1940-1948): the rows calErr(.., calCSV = true) appends
    // are kept in csv() instead of a file under savePath.
    void openCSV() { csv_open_ = true; }
    void closeCSV() {
        if (csv_open_) csv_ << "\n";
        csv_open_ = false;
    }
    const std::string csv() const { return csv_.str(); }
    // saveTime(ms, procedure) (h:1727-1744): "procedure: ms" records, kept in times()
    void saveTime(long ms, const std::string& procedure) { times_.push_back(procedure + ": " + std::to_string(ms)); }
    const std::vector<std::string>& times() const { return times_; }

    // calErr<T>(DP, DT, procedure, calCSV) (h:1748-1825): per region mask (nonocc, all, disc; empty
    // masks skipped) the bad ratio PBM (DP < 0 or |DT - DP| > errorThreshold) and the RMS, printed
    // like the reference and returned; the float arithmetic is sm_cal_err's (the reference's order).
    template <typename T = int16_t>
    std::vector<RegionErr> calErr(Mat& DP_, Mat& DT_, const std::string& procedure, bool calCSV = false) {
        static_assert(sizeof(T) == 2, "DP is CV_16S");
        if (DP_.empty() || DT_.empty() || DT_.depth() != CV_32F || DP_.rows != DT_.rows || DP_.cols != DT_.cols)
            throw std::invalid_argument("calErr: DP (CV_16S) and DT (CV_32F) of one size required");
        static const char* names[3] = {"nonocc", "all", "disc"};
        std::vector<RegionErr> out;
        const std::vector<int16_t> dp = DP_.packed<int16_t>();
        const std::vector<float> dt = DT_.packed<float>();
        for (int region = 0; region < 3; region++) {
            if (I_mask[region].empty()) continue;
            const std::vector<uint8_t> m = I_mask[region].packed<uint8_t>();
            RegionErr e{names[region], 0.f, 0.f};
            check(sm_cal_err(dp.data(), dt.data(), m.data(), DP_.rows, DP_.cols, (float)param_.errorThreshold, &e.PBM,
                             &e.RMS),
                  "calErr");
            std::cout << "\n" << e.region << "\terrorRatio: " << e.PBM << " epe: " << e.RMS << " " + procedure << "\n";
            if (calCSV && csv_open_) csv_ << e.PBM << ",";
            out.push_back(e);
        }
        return out;
    }
    std::vector<RegionErr> calErr() { return calErr<int16_t>(DP[0], DT, "DP0"); }

    Mat DP[2];        // int16 H x W disparity, -1 = invalid (h:2724)
    Mat DT;           // ground truth (cpp:2072)
    Mat I_mask[3];    // nonocc, all, disc (cpp:2073-2075)
    Parameters param_;
    int h_, w_, d_;
    sm_ctx* ctx_ = nullptr;

   private:
    bool refine_on_ = false, csv_open_ = false;
    std::ostringstream csv_;
    std::vector<std::string> times_;

    // a throwing constructor never runs the destructor: release the context (and its device
    // buffers) here before the exception leaves
    void init_or_release(const Mat& I1_c, const Mat& I2_c, const Mat& I1_g, const Mat& I2_g, int hip_device) {
        try {
            init(I1_c, I2_c, I1_g, I2_g, hip_device);
        } catch (...) {
            sm_destroy(ctx_);
            ctx_ = nullptr;
            throw;
        }
    }
    void init(const Mat& I1_c, const Mat& I2_c, const Mat& I1_g, const Mat& I2_g, int hip_device) {
        const Parameters& param = param_;
        if (I1_c.channels() != 3 || I2_c.channels() != 3 || I1_g.channels() != 1 || I2_g.channels() != 1 ||
            I1_c.depth() != CV_8U || I1_g.depth() != CV_8U)
            throw std::invalid_argument("expected BGR colour and single-channel gray u8 images");
        if (I2_c.rows != h_ || I2_c.cols != w_ || I1_g.rows != h_ || I1_g.cols != w_ || I2_g.rows != h_ ||
            I2_g.cols != w_ || I2_c.step != I1_c.step || I2_g.step != I1_g.step)
            throw std::invalid_argument("images of one size (and row stride per kind) required");
        sm_params p;
        sm_params_default(&p, param.numDisparities - 1, h_, w_);
        p.cost_method = costcalculation == "censusGrad" ? SM_COST_CENSUS_GRAD
                        : costcalculation == "Census"   ? SM_COST_CENSUS
                        : costcalculation == "ADCensus" ? SM_COST_AD_CENSUS
                        : costcalculation == "AD"       ? SM_COST_AD
                                                        : -1;
        if (p.cost_method < 0) throw std::invalid_argument("unsupported costcalculation: " + costcalculation);
        if (aggregation != "CBCA" && aggregation != "GF" && aggregation != "NL" && !aggregation.empty())
            throw std::invalid_argument("unsupported aggregation: " + aggregation);
        if (optimization != "sgm" && optimization != "so" && !optimization.empty())
            throw std::invalid_argument("unsupported optimization: " + optimization);
        p.aggregation = aggregation == "CBCA" ? SM_AGG_CBCA
                        : aggregation == "GF" ? SM_AGG_GF
                        : aggregation == "NL" ? SM_AGG_NL
                                              : SM_AGG_NONE;
        p.optimization = optimization == "sgm" ? SM_OPT_SGM : (optimization == "so" ? SM_OPT_SO : SM_OPT_WTA);
        p.census_ring = param.censusFunc == 3;
        p.lam_cen = (float)param.lamCen;
        p.lam_g = (float)param.lamG;
        const int sc = param.disSc > 1 ? param.disSc : 1;   // calArms: L / scale (cpp:5367-5371)
        p.arm_l = param.cbca_crossL0 / sc;
        p.arm_l_out = param.cbca_crossL_out0 / sc;
        p.arm_c_thresh = param.cbca_cTresh0;
        p.arm_c_thresh_out = param.cbca_cTresh_out0;
        p.arm_min_l = param.cbca_minArmL;
        p.cbca_iterations = param.cbca_iterationNum;
        p.sgm_paths = param.sgm_scanNum;
        p.sgm_cor_dif_thres = param.sgm_corDifThres;
        p.sgm_redu_coeff = param.sgm_reduCoeffi1;
        refine_on_ = Do_refine;
        p.do_refine = Do_refine ? 1 : 0;
        p.lr_max_diff = param.LRmaxDiff;
        p.disp_occ = param.DISP_OCC;
        p.region_vote_nums = param.region_vote_nums;
        p.do_region_vote = Do_regionVote ? 1 : 0;
        p.do_proper_ipol = Do_properIpol ? 1 : 0;
        p.do_last_median_blur = Do_lastMedianBlur ? 1 : 0;
        p.gf_mode = gf_my_guide ? SM_GF_MY_GUIDE : SM_GF_XIMGPROC;
        p.lr_consis = Do_LRConsis ? 1 : 0;
        check(sm_create(&ctx_, &p, hip_device), "sm_create");
        check(sm_set_images(ctx_, I1_c.data, I2_c.data, I1_c.step, I1_g.data, I2_g.data, I1_g.step), "sm_set_images");
    }
    void check(sm_status s, const char* what) {
        if (s != SM_OK)
            throw std::runtime_error(std::string(what) + ": " + (ctx_ ? sm_last_error(ctx_) : sm_status_string(s)));
    }
    friend void SolveAll(StereoMatching** smPyr, int PY_LVL, float REG_LAMBDA);
};

// SolveAll (cpp:2142-2208): PY_LVL = 1 scales vm[0]; PY_LVL in [2, 3] combines the levels
// smPyr[0..PY_LVL-1] of main_.cpp:134-156's pyramid into smPyr[0].
inline void SolveAll(StereoMatching** smPyr, int PY_LVL, float REG_LAMBDA) {
    if (PY_LVL == 1) {
        smPyr[0]->check(sm_solve_all(smPyr[0]->ctx_, PY_LVL, REG_LAMBDA), "SolveAll");
        return;
    }
    std::vector<sm_ctx*> lv;
    for (int i = 0; i < PY_LVL; i++) lv.push_back(smPyr[i]->ctx_);
    smPyr[0]->check(sm_solve_all_pyr(lv.data(), PY_LVL, REG_LAMBDA), "SolveAll");
}

}  // namespace smamd
