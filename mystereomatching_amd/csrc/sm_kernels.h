// sm_kernels.h — internal launch interface between the C-ABI layer and the kernels.
#pragma once
#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>

namespace sm {

enum { SM_M_CENSUS_GRAD = 0, SM_M_CENSUS = 1, SM_M_AD_CENSUS = 2, SM_M_AD = 3 };
enum { SGM_FIRST = 1, SGM_LAST = 2, SGM_KEEP = 4, SGM_SIGNED = 8 };  // KEEP: last path also writes the summed volume;
// SIGNED: costs may be negative (the guided filter's output), minima compare as floats
enum { CB_SCAN = 0, CB_NORM = 1, CB_NORM_SCAN = 2 };
constexpr int CBCA_TILE = 16;  // steps of lookahead per wave in the CBCA line sweeps

struct PrepArgs {
    const uint8_t* gray;        // [n][2][H][W]
    const uint8_t* bgr;         // [n][2][H][W][3]
    uint32_t* px;               // [n][2][H][W] packed BGR (written by the pack pass)
    uint32_t* pxh;              // [n][2][H][W] arm-walk words, horizontal flags (k_pack_arms)
    uint32_t* pxv;              // [n][2][H][W] arm-walk words, vertical flags
    ulonglong2* code;           // [n][2][H][W]
    uint8_t* arms;              // [n][view][plane][H][W] u32: plane 0 = L | R<<16, plane 1 = U | D<<16
    uint8_t* flags;             // [n][H][W] left image
    uint8_t* flags1;            // [n][H][W] right image (nullptr: not needed)
    int H, W, rv, ru, ring;
    int L, L_out, C_D, C_D_out, minL, cor_thres;
    int do_census, do_arms, do_flags;
    int pack_px;                // the packed-BGR plane px is read later (GF, so, refine)
};

struct CostArgs {
    float* vm;                  // [n][H][W][D] destination (view's volume)
    int seg;                    // pixels of a row per block (set by launch_cost: <= the LDS capacity)
    const ulonglong2* code;     // [n][2][H][W]
    const uint8_t* gray;        // [n][2][H][W] (censusGrad: the gradients, grad_at)
    const uint8_t* arms;        // [n][view][plane][H][W] u32: plane 0 = L | R<<16, plane 1 = U | D<<16
    const uint8_t* bgr;         // [n][2][H][W][3]
    int H, W, D, view, nwords;
    int cwords;                 // 32-bit census words in use: ceil(bits / 32)
    float census_default;       // codeLength * truncRat (h:938)
    float grad_trunc, grad_oor; // 500, sqrt(2*500^2) (cpp:440)
    int grad_adaptive;
    float lam2;                 // lamG
    float ad_trunc;             // "AD" method truncation
    float ad_oor_exp;           // ADCensus: expf(-(trunc)/lamAD) for out-of-range pairs
    const float* lut;           // the context's exponent tables [2][1024]: expf(-x / lam) of the
                                // census (or AD-census census) term, then the ADCensus AD term
};

struct CbcaArgs {
    float* vm;                  // [n][H][W][D], in place
    float* dummy;               // 64 floats: private slots for lanes past D
    const uint32_t* arms;       // [n][view][plane][H][W]: plane 0 = L | R<<16, plane 1 = U | D<<16
    const float* vm_end;        // end of the volume allocation (reads past it return 0)
    const uint32_t* arms_end;   // end of the arm allocation (which has a 2 * lag row front pad)
    int H, W, D;
    int lag;                    // max arm length (the ring size is derived in sm_cbca.hip)
    int apply_scale;
    float scale;                // SolveAll weight (fused into the last normalising pass)
    int view;                   // 0: vm[0] (left reference), 1: vm[1] (right reference, Do_refine)
    int num_cu;                 // compute units of the device
    int arm_pad_rows;           // rows of front pad before the arm planes (2 lag; the allocation also
                                // has >= 2 lag + 64 rows of tail pad, and the volumes >= 8 rows)
    int div_safe;               // 1: every dividend of this launch's normalisation is 0 or >= 2^-110
                                // (proven by the host, cbca_div_safe): the area division needs no check
};
constexpr int CBCA_VM_TAIL_ROWS = 8;   // volume tail pad in rows of W * D floats (fast V sweeps)

struct SgmArgs {
    float* vm;                  // [n][H][W][D] aggregated costs (also the final volume if keep_final)
    float* acc;                 // [n][H][W][D] running path sum
    float* dummy;               // 64 floats: store target of elements past D
    const uint8_t* bgr;         // [n][2][H][W][3] (left colour used for P1/P2 adaptivity)
    int16_t* disp;              // [n][H][W]
    const uint8_t* flags;       // [n][H][W] bit i: colour-difference penalty towards direction i
    int H, W, D, rv, ru, dir;
    float p1, p2;
    int cor_thres, redu, keep_final;
    int signed_costs;           // 1: C may be < 0 (aggregation GF): k_sgm with float minima
    int n;                      // pairs in the launch
    // checkpointed path pairs (k_sgm_ck): the second path of the pair is the first one reversed
    float* ck;                  // [n][lines][segments][D]: the first path's L at segment ends
    int dir2;                   // direction index of the pair's second path
    const float* lx;            // CK_X: [n][H][W][D] L of the path between the pair's two (8 paths: L5)
};

struct GfPix {                  // guided filter, p-independent terms of one pixel (sm_gf.hip)
    double cof[9];              // the nine cofactor expressions of guideFilterCore_matlab (cpp:5060-5078)
    double idet;                // 1 / DET
    float N;                    // BoxFilter(ones)
    float mI[3];                // mean_I[c], BGR
};

struct GfArgs {
    float* vm;                  // [n][H][W][D], filtered in place
    float *s0, *s1, *s2, *s3;   // four scratch volumes [n][H][W][D]
    const uint8_t* bgr;         // the view's colour image of pair 0 ([n][2][H][W][3] + view offset)
    size_t bgr_pair_stride;     // bytes between pairs
    const uint32_t* px;         // the same image as packed B | G << 8 | R << 16 words (prep's k_pack_bgr)
    size_t px_pair_stride;      // words between pairs
    float* planes;              // [n][10][H][W] scratch
    GfPix* pix;                 // [n][H][W]
    int H, W, D;
    float eps;
    int solve_all;              // 1: the output is SolveAll's `0 + w * q` (cpp:2189-2201), w = scale
    float scale;
};
void launch_gf(const GfArgs& a, int n, hipStream_t st);

struct GfCvArgs {               // guided filter, ximgproc form (sm_gf_cv.hip); pair-relative bases
    float* vm;                  // [n][H][W][D], filtered in place
    double* rs;                 // row sums: 4 channel planes, plane c at rs + c * cap * nvol
    float* ab;                  // alpha_0..2, beta: 4 planes, plane c at ab + c * cap * nvol
    int cap;                    // pairs per channel plane (the context's batch capacity)
    const uint32_t* px;         // the view's packed B | G << 8 | R << 16 words of pair 0
    size_t px_pair_stride;      // words between pairs
    double* img_rs;             // [n][9][H][W] image-plane row sums
    float* pix;                 // [n][9][H][W] mean_I (3), Sigma^-1 (6)
    int H, W, D;
    float eps;
    int solve_all;              // 1: the output is SolveAll's `0 + w * q` (cpp:2189-2201), w = scale
    float scale;
};
void launch_gf_cv(const GfCvArgs& a, int n, hipStream_t st);

struct NlArgs {                 // non-local tree filter (sm_nl.hip); node ids = pair * H W + pixel
    const int4* rec;            // path nodes, each path bottom -> top: {x, meta, child weights, parent}
                                //   meta = nchild | (heavy + 1) << 3 | child directions << 6 (2 bits
                                //   each: +1, -1, +W, -W) | own edge weight << 16
    const int* chain_start;     // first record of each path
    const int* chain_len;
    const int* order_up;        // path indices sorted by up round
    const int* order_down;      // path indices sorted by down round
    const double* table;        // exp(-i / (255 sigma)), i = 0..255
    double* val;                // [nodes][D] up sums, then final values (in place)
    float* vm;                  // [nodes][D] normalised aggregated costs out
    const float* vc;            // [nodes][D] costs in (vm itself, or the pipelined front's volume)
    int solve_all;              // 1: vm out is SolveAll's `0 + w * v` (cpp:2189-2201), w = scale
    float scale;
    double* oup;                // [nodes] the ones volume's up sums (qx_tree_filter on ones)
    double* ofin;               // [nodes] its final sums: the normaliser fin(1)
    long nodes;                 // n H W
    int W;
};
constexpr int NL_REC_PAD = 64;  // zero records after the last path (blocked reads past a path's end)
constexpr int NL_LEVELS = 32;   // round tables of the GPU tree walk (light depth <= log2(H W) < 32)
// The tree walk on the GPU (sm_nl_walk.hip): from the neighbour words adj [n H W] of the spanning
// trees, the path records rec [n H W] (bottom -> top per path), chain_start / chain_len per path
// (indexed by the path top's preorder position), the paths of every up / down round (order_up,
// order_down) and offs [2 (NL_LEVELS + 1) + 1]: up round offsets, down round offsets, error flags.
size_t nl_walk_scratch_bytes(int H, int W, int n);
void launch_nl_walk(const uint32_t* adj, int H, int W, int n, uint8_t* scratch, int4* rec, int* chain_start, int* chain_len,
                    int* order_up, int* order_down, int* offs, hipStream_t st);
void launch_nl_edges(const uint8_t* bgr, size_t pair_stride, uint8_t* med, uint8_t* ew, int H, int W, int n, hipStream_t st);
void launch_nl_round(const NlArgs& a, bool up, int lo, int hi, int P, hipStream_t st);
// minimum spanning trees of n pairs' edge weights (sm_nl_mst.hip): par / best [n H W] and
// scratch [nl_mst_scratch_bytes] work space; adj [n H W] the neighbour words of
// nl_tree_from_lists (sm_nl_tree.h)
size_t nl_mst_scratch_bytes(int H, int W, int n);
void launch_nl_mst(const uint8_t* ew, int H, int W, int n, int* par, unsigned long long* best, uint8_t* scratch,
                   uint32_t* adj, hipStream_t st);

struct SoArgs {                 // scan-line optimisation "so" (sm_so.hip)
    float* vm;                  // [n][H][W][D] costs (accumulated in place when keep_final)
    uint8_t* trace;             // [n][H][W][D] choice codes
    uint16_t* cidx;             // [n][H][W] row-minimum index of the previous column
    const uint32_t* px;         // [n][2][H][W] packed BGR (view 0 = I_c[0] is used)
    int16_t* disp;              // [n][H][W]
    int H, W, D, n, keep_final;
};

constexpr int kMaxPyr = 8;      // PY_LVL limit (sm_solve_all_pyr)
struct PyrArgs {                // SolveAll over PY_LVL pyramid levels (sm_pyramid.hip)
    float* vm[kMaxPyr];         // level s volume [n][H_s][W_s][D_s]; vm[0] is updated in place
    int H[kMaxPyr], W[kMaxPyr], D[kMaxPyr];
    float w[kMaxPyr];           // invWgt[s] = regInv(0, s)
    int levels, n;
};

void launch_cost(const CostArgs& a, int method, int n, hipStream_t st);
void launch_prep(const PrepArgs& a, int n, hipStream_t st);
size_t prep_smem_bytes(int rv, int ru, int L_out);
void launch_cbca(const CbcaArgs& a, bool horiz, int mode, int n, hipStream_t st);
void launch_scale(float* vm, size_t n, float w, hipStream_t st);
void launch_sgm_path(const SgmArgs& a, int mode, int n, hipStream_t st);
// Checkpointed path pairs (sm_sgm.hip, k_sgm_ck): CK_A sweeps the pair's first path and keeps
// its L every sgm_ck_seg(D) steps; CK_B sweeps the second path, recomputing the first one's L
// segment by segment from those checkpoints, and writes L_first + L_second (CK_B), adds both to
// the running sum (CK_B | CK_MID, 8 paths) or adds them, takes the WTA and writes the map
// (CK_B | SGM_LAST [| SGM_KEEP]).
// CK_B | CK_MID | CK_X (8 paths, the diagonal pair (4, 6)): acc = ((acc + L4) + L5) + L6 with L5
// read from SgmArgs::lx (a path-5 sweep in SGM_FIRST mode stored it there).
enum { CK_A = 16, CK_B = 32, CK_MID = 64, CK_X = 128 };
bool sgm_ck_ok(int D, int paths);
int sgm_ck_seg(int D);
bool sgm_ck_diag_ok(int D, int paths);   // 8 paths: the diagonal pair (4, 6) checkpointed as well
int sgm_ck_diag_seg();
void launch_sgm_ck(const SgmArgs& a, int mode, int n, hipStream_t st);
void launch_wta(const float* vm, int16_t* disp, int n, int H, int W, int D, hipStream_t st);
void launch_expf_range(uint32_t first, uint32_t n, float* out, hipStream_t st);
void launch_copy_x4(const void* in, void* out, size_t bytes, int grid, hipStream_t st);   // bytes % 16384 == 0
void launch_div_check(int exp2, int bmax, unsigned long long* bad, hipStream_t st);
float expf_host(float x);
// refinement (sm_refine.hip)
void launch_lr_check(int16_t* d0, const int16_t* d1, int n, int H, int W, float maxdiff, hipStream_t st);
void launch_region_vote(const int16_t* src, int16_t* dst, const uint32_t* arms, int n, int H, int W, int rv_s,
                        float rv_ratio, hipStream_t st);
void launch_proper_ipol(const int16_t* src, int16_t* dst, const uint32_t* px, int n, int H, int W, int disp_occ,
                        hipStream_t st);
void launch_so(const SoArgs& a, hipStream_t st);
void launch_pyr_down(const uint8_t* src, uint8_t* dst, int rows, int cols, int ch, hipStream_t st);
void launch_pyr_down_f32(const float* src, float* dst, int rows, int cols, hipStream_t st);
void launch_solve_all_pyr(const PyrArgs& a, hipStream_t st);
void launch_median3(const int16_t* src, int16_t* dst, int n, int H, int W, hipStream_t st);
int sgm_k_for(int D);

}  // namespace sm
