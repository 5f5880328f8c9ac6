// main_shaped.cpp — the reference driver main_.cpp:15-19 and 85-178, with OpenCV's Mat / imread /
// pyrDown taken from include/stereo_matching.hpp (`using namespace smamd` where main_ has `using
// namespace cv`) and the dataset paths taken from argv.  Test program (tests/test_cpp_facade.py):
// it must compile unchanged against the facade, and on a GPU its DP[0] must equal the oracle's.
// Usage: main_shaped IMGDIR MAXDISP REDUCE_COEFF OUT.i16
//   IMGDIR holds a Middlebury-2003-style object folder as main_.cpp reads it (teddy / cones
//   entries of main:33-39): im2.png im6.png disp2.png all.png nonocc.png disc.png;
//   OUT.i16 receives DP[0] as raw little-endian int16, rows x cols.
#include "stereo_matching.hpp"

#include <iostream>

using namespace std;
using namespace smamd;

string StereoMatching::costcalculation = "censusGrad";   // main_.cpp:15
string StereoMatching::aggregation = "CBCA";              // main_.cpp:16
string StereoMatching::optimization = "sgm";              // main_.cpp:17
string StereoMatching::object = "";                       // main_.cpp:18
const string StereoMatching::root = "";                   // main_.cpp:19

int main(int argc, char* argv[]) {
    if (argc < 5) {
        cout << "usage: " << argv[0] << " IMGDIR MAXDISP REDUCE_COEFF OUT.i16" << endl;
        return 2;
    }
    const string method = StereoMatching::costcalculation + StereoMatching::aggregation + StereoMatching::optimization;
    printf("method: %s\n", method.c_str());
    const string imgroot = string(argv[1]) + "/";
    vector<int> maxdispList = {atoi(argv[2])};
    vector<float> disp_reduceCoeffList = {(float)atof(argv[3])};
    const int i = 0;
    string dataset = "MD";

    // main_.cpp:26-39, 85-129 (leftNameList / rightNameList / dispNameList of teddy and cones)
    string all_maskN = "all.png";
    string nonocc_maskN = "nonocc.png";
    string disc_maskN = "disc.png";
    string leftimg = imgroot + "im2" + ".png";
    string rightimg = imgroot + "im6" + ".png";
    string img_disp = imgroot + "disp2" + ".png";
    string all_mask = imgroot + all_maskN;
    string nonocc_mask = imgroot + nonocc_maskN;
    string disc_mask = imgroot + disc_maskN;
    Mat I1_c = imread(leftimg, 1);
    Mat I2_c = imread(rightimg, 1);
    Mat I1 = imread(leftimg, 0);
    Mat I2 = imread(rightimg, 0);
    Mat all_maskM = imread(all_mask, 0);
    Mat nonocc_maskM = imread(nonocc_mask, 0);
    Mat disc_maskM = imread(disc_mask, 0);
    Mat DT = imread(img_disp, 0);
    if (I1.empty() || I2.empty() || I1_c.empty() || I2_c.empty()) {
        cout << "can't read original img" << endl;
        return -1;
    }
    if (all_maskM.empty() || nonocc_maskM.empty() || disc_maskM.empty()) {
        cout << "can't read mask img" << endl;
    }
    std::cout << "read-in img done" << endl;
    if (StereoMatching::preMedBlur) return 3;   // cv::medianBlur on the inputs (main:120-124): not used
    if (dataset == "KT") DT.convertTo(DT, CV_32F, 1.0 / 256);
    if (dataset == "MD") DT.convertTo(DT, CV_32F, 1.0 / disp_reduceCoeffList[i]);

    // main_.cpp:131-178
    int lamG = 1, lamCen = 13, M = 2, lamc = 109, ts = 10;
    string errCsvName = "test.csv";
    int disSc = 1;
    int PY_LEV = 1;
    StereoMatching** smPsy = new StereoMatching*[PY_LEV];
    clock_t start = clock();
    for (int p = 0; p < PY_LEV; p++) {
        printf("\n\tPyramid: %d:", p);
        StereoMatching::Parameters param(maxdispList[i], I1_c.rows, I1_c.cols, lamCen, lamG, M, lamc, ts, errCsvName, disSc);
        smPsy[p] = new StereoMatching(I1_c, I2_c, I1, I2, DT, all_maskM, nonocc_maskM, disc_maskM, param);
        smPsy[p]->costCalculate();

        maxdispList[i] = maxdispList[i] / 2 + 1;
        disSc *= 2;
        pyrDown(I1_c, I1_c);
        pyrDown(I2_c, I2_c);
        pyrDown(I1, I1);
        pyrDown(I2, I2);
        pyrDown(DT, DT);
        pyrDown(all_maskM, all_maskM);
        if (nonocc_maskM.data) pyrDown(nonocc_maskM, nonocc_maskM);
        if (disc_maskM.data) pyrDown(disc_maskM, disc_maskM);
    }
    const auto t1 = std::chrono::system_clock::now();
    (void)t1;
    float REG_LAMBDA = 0.3;  // 0.3 for middlebury
    SolveAll(smPsy, PY_LEV, REG_LAMBDA);
    smPsy[0]->openCSV();
    smPsy[0]->dispOptimize();
    if (StereoMatching::Do_refine) smPsy[0]->refine();
    smPsy[0]->closeCSV();
    clock_t end = clock();
    clock_t time = end - start;
    smPsy[0]->saveTime(time, "all");
    cout << "all Time: " << time << endl;

    // the result (public member DP[0], h:2724) and the evaluator over the stored DT / masks
    smPsy[0]->calErr();
    {
        ofstream o(argv[4], ios::binary);
        const Mat& dp = smPsy[0]->DP[0];
        for (int v = 0; v < dp.rows; v++) o.write((const char*)dp.ptr<int16_t>(v), (streamsize)dp.cols * 2);
    }

    for (int p = 0; p < PY_LEV; p++) {
        delete smPsy[p];
        smPsy[p] = NULL;
    }
    delete[] smPsy;
    smPsy = NULL;
    cout << "complete " << StereoMatching::object << endl;
    return 0;
}
