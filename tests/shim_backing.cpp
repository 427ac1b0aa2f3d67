// shim_backing.cpp -- TEST INFRASTRUCTURE for tests/pose_driver.cpp: minimal definitions of the
// reference symbols the drop-in shim (integration/openpose_hip_shim.cpp, arrayCpuGpuHip.cpp) links
// against, written here because the reference's own definitions live in files that need OpenCV
// (core/array.cpp, core/matrix.cpp) or would put reference-built code on the GPU box (no
// reference code travels).  Each follows the contract of the declaration in the reference header
// it implements; none of them is product code.
//   op::error                      utilities/errorAndLog.hpp  (throws, as the reference's does after logging)
//   op::Matrix::Matrix()           core/matrix.hpp            (empty wrapper; Array keeps one)
//   op::Point<int>                 core/point.hpp             (plain x, y)
//   op::Array<T>                   core/array.hpp             (shared buffer, fast copies)
//   op::PoseExtractorNet           pose/poseExtractorNet.hpp  (properties, thread check, results)
//   op::getPose* / addBkgChannel   pose/poseParameters.hpp    (from libopk's tables, which are
//                                  generated from poseParameters.cpp and pinned by the tests)
#include <cstring>
#include <stdexcept>
#include <string>
#include <thread>
#include <vector>

#include <openpose/core/array.hpp>
#include <openpose/core/matrix.hpp>
#include <openpose/core/point.hpp>
#include <openpose/pose/poseExtractorNet.hpp>
#include <openpose/pose/poseParameters.hpp>
#include <openpose/utilities/errorAndLog.hpp>

#include "opk.h"

namespace op
{
    void error(const std::string& message, const int line, const std::string& function, const std::string& file)
    {
        throw std::runtime_error(message + " (" + file + ":" + std::to_string(line) + " " + function + ")");
    }

    Matrix::Matrix() {}

    // ---- Point ----------------------------------------------------------------------------------
    template <typename T> Point<T>::Point(const T x_, const T y_) : x{x_}, y{y_} {}
    template <typename T> Point<T>::Point(const Point<T>& p) : x{p.x}, y{p.y} {}
    template <typename T> Point<T>& Point<T>::operator=(const Point<T>& p) { x = p.x; y = p.y; return *this; }
    template <typename T> Point<T>::Point(Point<T>&& p) : x{p.x}, y{p.y} {}
    template <typename T> Point<T>& Point<T>::operator=(Point<T>&& p) { x = p.x; y = p.y; return *this; }
    template struct Point<int>;
    template struct Point<float>;
    template struct Point<double>;

    // ---- Array: a shared buffer; copies share it (array.hpp "fast copy") ------------------------
    template <typename T> void Array<T>::resetAuxiliary(const std::vector<int>& sizes, T* const dataPtr)
    {
        mSize = sizes;
        mVolume = 1;
        for (const auto s : sizes)
            mVolume *= (size_t)s;
        if (sizes.empty())
            mVolume = 0;
        if (dataPtr)
            spData.reset(dataPtr, [](T*) {});
        else if (mVolume > 0)
            spData.reset(new T[mVolume](), std::default_delete<T[]>());
        else
            spData.reset();
        pData = spData.get();
    }
    template <typename T> Array<T>::Array(const int size) : mVolume{0}, pData{nullptr} { reset(size); }
    template <typename T> Array<T>::Array(const std::vector<int>& sizes) : mVolume{0}, pData{nullptr} { reset(sizes); }
    template <typename T> Array<T>::Array(const std::vector<int>& sizes, const T value) : mVolume{0}, pData{nullptr}
    {
        reset(sizes, value);
    }
    template <typename T> Array<T>::Array(const Array<T>& a) :
        mSize{a.mSize}, mVolume{a.mVolume}, spData{a.spData}, pData{a.pData}, mCvMatData{a.mCvMatData} {}
    template <typename T> Array<T>& Array<T>::operator=(const Array<T>& a)
    {
        mSize = a.mSize; mVolume = a.mVolume; spData = a.spData; pData = a.pData;
        return *this;
    }
    template <typename T> Array<T>::Array(Array<T>&& a) :
        mSize{std::move(a.mSize)}, mVolume{a.mVolume}, spData{std::move(a.spData)}, pData{a.pData},
        mCvMatData{a.mCvMatData}
    {
        a.mVolume = 0;
        a.pData = nullptr;
    }
    template <typename T> Array<T>& Array<T>::operator=(Array<T>&& a)
    {
        mSize = std::move(a.mSize); mVolume = a.mVolume; spData = std::move(a.spData); pData = a.pData;
        a.mVolume = 0;
        a.pData = nullptr;
        return *this;
    }
    template <typename T> void Array<T>::reset(const int size)
    {
        resetAuxiliary(size > 0 ? std::vector<int>{size} : std::vector<int>{});
    }
    template <typename T> void Array<T>::reset(const std::vector<int>& sizes) { resetAuxiliary(sizes); }
    template <typename T> void Array<T>::reset(const std::vector<int>& sizes, const T value)
    {
        resetAuxiliary(sizes);
        for (size_t i = 0; i < mVolume; i++)
            pData[i] = value;
    }
    template <typename T> int Array<T>::getSize(const int index) const
    {
        return index >= 0 && index < (int)mSize.size() ? mSize[index] : 0;
    }
    template <typename T> T& Array<T>::commonAt(const int index) const
    {
        if (index < 0 || (size_t)index >= mVolume)
            error("Index out of bounds.", __LINE__, __FUNCTION__, __FILE__);
        return pData[index];
    }
#define OPK_ARRAY_MEMBERS(T)                                                                   \
    template Array<T>::Array(const int);                                                       \
    template Array<T>::Array(const std::vector<int>&);                                         \
    template Array<T>::Array(const std::vector<int>&, const T);                                \
    template Array<T>& Array<T>::operator=(const Array<T>&);                                   \
    template Array<T>::Array(Array<T>&&);                                                      \
    template Array<T>& Array<T>::operator=(Array<T>&&);                                        \
    template void Array<T>::reset(const int);                                                  \
    template void Array<T>::reset(const std::vector<int>&);                                    \
    template void Array<T>::reset(const std::vector<int>&, const T);                           \
    template int Array<T>::getSize(const int) const;                                           \
    template T& Array<T>::commonAt(const int) const;
    OPK_ARRAY_MEMBERS(float)
    OPK_ARRAY_MEMBERS(double)
#undef OPK_ARRAY_MEMBERS
    // the copy constructor cannot be named in an explicit instantiation (the converting
    // constructor template of array.hpp:96 makes it ambiguous): instantiated by use
    __attribute__((used)) void opkBackingInstantiateArrayCopies(Array<float>& f, Array<double>& d)
    {
        Array<float> f2{f};
        Array<double> d2{d};
        f = f2;
        d = d2;
    }

    // ---- pose parameters through libopk's generated tables ------------------------------------
    unsigned int getPoseNumberBodyParts(const PoseModel poseModel)
    {
        int parts = 0;
        if (opk_pose_model_info((int)poseModel, &parts, nullptr, nullptr, nullptr, nullptr, nullptr) != OPK_OK)
            error(opk_last_error(), __LINE__, __FUNCTION__, __FILE__);
        return (unsigned)parts;
    }
    bool addBkgChannel(const PoseModel poseModel)
    {
        int bkg = 0;
        if (opk_pose_model_info((int)poseModel, nullptr, &bkg, nullptr, nullptr, nullptr, nullptr) != OPK_OK)
            error(opk_last_error(), __LINE__, __FUNCTION__, __FILE__);
        return bkg != 0;
    }
    const std::vector<unsigned int>& getPoseMapIndex(const PoseModel poseModel)
    {
        static thread_local std::vector<unsigned int> idx;
        int parts = 0, bkg = 0, channels = 0;
        if (opk_pose_model_info((int)poseModel, &parts, &bkg, nullptr, &channels, nullptr, nullptr) != OPK_OK)
            error(opk_last_error(), __LINE__, __FUNCTION__, __FILE__);
        std::vector<int> m(channels - parts - bkg);
        if (opk_pose_model_info((int)poseModel, nullptr, nullptr, nullptr, nullptr, nullptr, m.data()) != OPK_OK)
            error(opk_last_error(), __LINE__, __FUNCTION__, __FILE__);
        idx.assign(m.begin(), m.end());
        return idx;
    }
    float getPoseNetDecreaseFactor(const PoseModel poseModel) { return poseModel != PoseModel::BODY_19_X2 ? 8.f : 4.f; }
    const std::string& getPoseProtoTxt(const PoseModel)
    {
        static const std::string s = "builtin:BODY_25";
        return s;
    }
    const std::string& getPoseTrainedModel(const PoseModel)
    {
        static const std::string s = "";
        return s;
    }

    // ---- PoseExtractorNet: the base-class state the extractor fills and the Wrapper reads -------
    PoseExtractorNet::PoseExtractorNet(const PoseModel poseModel, const std::vector<HeatMapType>& heatMapTypes,
                                       const ScaleMode heatMapScaleMode, const bool addPartCandidates,
                                       const bool maximizePositives) :
        mPoseModel{poseModel}, mNetOutputSize{0, 0}, mScaleNetToOutput{-1.f}, mHeatMapTypes{heatMapTypes},
        mHeatMapScaleMode{heatMapScaleMode}, mAddPartCandidates{addPartCandidates}
    {
        // BODY_25 defaults (poseParameters.cpp), maximizePositives' alternatives
        mProperties[(int)PoseProperty::NMSThreshold] = maximizePositives ? 0.02 : 0.05;
        mProperties[(int)PoseProperty::ConnectInterMinAboveThreshold] = maximizePositives ? 0.75 : 0.95;
        mProperties[(int)PoseProperty::ConnectInterThreshold] = maximizePositives ? 0.01 : 0.05;
        mProperties[(int)PoseProperty::ConnectMinSubsetCnt] = maximizePositives ? 2 : 3;
        mProperties[(int)PoseProperty::ConnectMinSubsetScore] = maximizePositives ? 0.05 : 0.4;
    }
    PoseExtractorNet::~PoseExtractorNet() {}
    void PoseExtractorNet::initializationOnThread()
    {
        mThreadId = std::this_thread::get_id();
        netInitializationOnThread();
    }
    Array<float> PoseExtractorNet::getPoseKeypoints() const { return mPoseKeypoints; }
    Array<float> PoseExtractorNet::getPoseScores() const { return mPoseScores; }
    float PoseExtractorNet::getScaleNetToOutput() const { return mScaleNetToOutput; }
    double PoseExtractorNet::get(const PoseProperty property) const { return mProperties.at((int)property); }
    void PoseExtractorNet::set(const PoseProperty property, const double value) { mProperties.at((int)property) = value; }
    void PoseExtractorNet::checkThread() const
    {
        if (mThreadId != std::this_thread::get_id())
            error("The CPU/GPU pointer data cannot be accessed from a different thread.", __LINE__, __FUNCTION__,
                  __FILE__);
    }
}
