// arrayCpuGpuHip.cpp -- op::ArrayCpuGpu<T> on HIP memory through libopk_hip.so (replaces
// src/openpose/core/arrayCpuGpu.cpp, which is a Caffe-Blob wrapper and errors in every
// constructor without USE_CAFFE, arrayCpuGpu.cpp:23-40).
//
// The reference class (include/openpose/core/arrayCpuGpu.hpp:14-106) is a PIMPL over caffe::Blob;
// here its ImplArrayCpuGpu restates the Blob + SyncedMemory contract the reference's callers rely
// on, with device memory from opk_malloc on the calling thread's libopk context (the shim's, so it
// shares the GPU that thread's NetHip / extractors use):
//   * shape, count, CanonicalAxisIndex, LegacyShape (1 past the last axis), offset, shape_string
//     ("n c h w (count)") -- caffe/blob.hpp;
//   * data and diff are two synced buffers: UNINITIALIZED -> (cpu_data: zeroed host) or (gpu_data:
//     zeroed device); a read on the side that is behind copies from the head side and leaves both
//     SYNCED; mutable_* moves the head to that side; set_cpu_data / set_gpu_data adopt an external
//     buffer as the head (not owned) -- caffe/syncedmem.cpp;
//   * Reshape keeps the buffers while the count fits the capacity, reallocates (contents dropped)
//     otherwise -- Blob::Reshape;
//   * Update = data - diff, asum / sumsq / scale on the host copy (Caffe's math on the head side;
//     same values up to the float summation order).
// The Caffe-blob constructor has nothing to wrap here and raises op::error.
#include <algorithm>
#include <cmath>
#include <cstring>
#include <sstream>
#include <vector>

#include <openpose/core/arrayCpuGpu.hpp>
#include <openpose/utilities/errorAndLog.hpp>

#include "opk.h"
#include "opk_shim.hpp"

namespace op
{
    namespace
    {
        void checkOpk(const int rc, const int line, const char* function)
        {
            if (rc != OPK_OK)
                error(std::string{"libopk_hip: "} + opk_last_error(), line, function, __FILE__);
        }

        // caffe::SyncedMemory on libopk device memory
        class SyncedHip
        {
        public:
            enum Head { UNINITIALIZED, HEAD_AT_CPU, HEAD_AT_GPU, SYNCED };
            explicit SyncedHip(const size_t bytes) : mBytes{bytes} {}
            ~SyncedHip()
            {
                if (mOwnGpu && mGpu)
                    opk_free(mCtx.get(), mGpu);
            }
            SyncedHip(const SyncedHip&) = delete;
            SyncedHip& operator=(const SyncedHip&) = delete;

            const void* cpu() { toCpu(); return cpuPtr(); }
            const void* gpu() { toGpu(); return mGpu; }
            void* mutableCpu() { toCpu(); mHead = HEAD_AT_CPU; return cpuPtr(); }
            void* mutableGpu() { toGpu(); mHead = HEAD_AT_GPU; return mGpu; }
            // an adopted (external) buffer holds `bytes` = the blob's current count, which may be less
            // than this memory's capacity after a shrinking Reshape: transfers are limited to it
            void setCpu(void* data, const size_t bytes)
            {
                if (data == nullptr)
                    error("set_cpu_data: NULL pointer.", __LINE__, __FUNCTION__, __FILE__);
                mOwnCpu.clear();
                mCpu = data;
                mExtBytes = std::min(bytes, mBytes);
                mHead = HEAD_AT_CPU;
            }
            void setGpu(void* data, const size_t bytes)
            {
                if (data == nullptr)
                    error("set_gpu_data: NULL pointer.", __LINE__, __FUNCTION__, __FILE__);
                if (mOwnGpu && mGpu)
                    opk_free(mCtx.get(), mGpu);
                mCtx = opkShimThreadContext();
                mGpu = data;
                mOwnGpu = false;
                mExtBytes = std::min(bytes, mBytes);
                mHead = HEAD_AT_GPU;
            }
            size_t bytes() const { return mBytes; }

        private:
            void* cpuPtr() { return mCpu ? mCpu : (void*)mOwnCpu.data(); }
            size_t xfer() const { return mCpu || (mGpu && !mOwnGpu) ? mExtBytes : mBytes; }
            void allocCpu()
            {
                if (!mCpu && mOwnCpu.size() != mBytes)
                    mOwnCpu.assign(mBytes, 0);
            }
            void allocGpu()
            {
                if (mGpu)
                    return;
                mCtx = opkShimThreadContext();
                checkOpk(opk_malloc(mCtx.get(), &mGpu, std::max<size_t>(mBytes, 1)), __LINE__, __FUNCTION__);
                mOwnGpu = true;
            }
            void toCpu()
            {
                switch (mHead)
                {
                    case UNINITIALIZED:
                        allocCpu();
                        std::memset(cpuPtr(), 0, mBytes);
                        mHead = HEAD_AT_CPU;
                        break;
                    case HEAD_AT_GPU:
                        allocCpu();
                        if (xfer())
                            checkOpk(opk_memcpy_d2h(mCtx.get(), cpuPtr(), mGpu, xfer()), __LINE__, __FUNCTION__);
                        mHead = SYNCED;
                        break;
                    default:
                        break;
                }
            }
            void toGpu()
            {
                switch (mHead)
                {
                    case UNINITIALIZED:
                        allocGpu();
                        checkOpk(opk_memset(mCtx.get(), mGpu, 0, mBytes), __LINE__, __FUNCTION__);
                        mHead = HEAD_AT_GPU;
                        break;
                    case HEAD_AT_CPU:
                        allocGpu();
                        if (xfer())
                            checkOpk(opk_memcpy_h2d(mCtx.get(), mGpu, cpuPtr(), xfer()), __LINE__, __FUNCTION__);
                        mHead = SYNCED;
                        break;
                    default:
                        break;
                }
            }

            const size_t mBytes;
            Head mHead = UNINITIALIZED;
            std::vector<unsigned char> mOwnCpu;
            void* mCpu = nullptr;   // external host buffer (set_cpu_data), else mOwnCpu
            size_t mExtBytes = 0;   // bytes of an adopted buffer
            OpkContext mCtx;   // the context of the device buffer (kept alive by this)
            void* mGpu = nullptr;
            bool mOwnGpu = false;
        };
    }

    template<typename T>
    struct ArrayCpuGpu<T>::ImplArrayCpuGpu
    {
        std::vector<int> shape;
        int count = 0;
        int capacity = 0;
        std::unique_ptr<SyncedHip> data, diff, shapeData;

        void reshape(const std::vector<int>& newShape)
        {
            if (newShape.size() > 32)   // kMaxBlobAxes (caffe/blob.hpp)
                error("Too many axes.", __LINE__, __FUNCTION__, __FILE__);
            long long c = 1;
            for (const auto d : newShape)
            {
                if (d < 0)
                    error("Negative blob dimension.", __LINE__, __FUNCTION__, __FILE__);
                c *= d;
                if (c > 0x7fffffffLL)
                    error("Blob size exceeds INT_MAX.", __LINE__, __FUNCTION__, __FILE__);
            }
            shape = newShape;
            count = (int)c;
            shapeData.reset(new SyncedHip{newShape.size() * sizeof(int)});
            if (!newShape.empty())
                std::memcpy(shapeData->mutableCpu(), newShape.data(), newShape.size() * sizeof(int));
            if (count > capacity || !data)
            {
                capacity = count;
                data.reset(new SyncedHip{(size_t)capacity * sizeof(T)});
                diff.reset(new SyncedHip{(size_t)capacity * sizeof(T)});
            }
        }
    };

    template<typename T>
    ArrayCpuGpu<T>::ArrayCpuGpu() : spImpl{std::make_shared<ImplArrayCpuGpu>()}
    {
    }

    template<typename T>
    ArrayCpuGpu<T>::ArrayCpuGpu(const void* caffeBlobTPtr)
    {
        (void)caffeBlobTPtr;
        error("ArrayCpuGpu: no Caffe blob to wrap in the HIP build (libopk_hip owns its buffers).",
              __LINE__, __FUNCTION__, __FILE__);
    }

    template<typename T>
    ArrayCpuGpu<T>::ArrayCpuGpu(const Array<T>& array, const bool copyFromGpu)
        : spImpl{std::make_shared<ImplArrayCpuGpu>()}
    {
        try
        {
            // arrayCpuGpu.cpp:78-100: a 3-D Array gets a leading batch of 1
            std::vector<int> arraySize;
            if (array.getNumberDimensions() == 3)
                arraySize.emplace_back(1);
            for (const auto& sizeI : array.getSize())
                arraySize.emplace_back(sizeI);
            spImpl->reshape(arraySize);
            if (!copyFromGpu)
            {
                const auto* const arrayPtr = array.getConstPtr();
                std::copy(arrayPtr, arrayPtr + array.getVolume(),
                          static_cast<T*>(spImpl->data->mutableCpu()));
            }
            else
                error("Not implemented yet. Let us know you are interested on this function.",
                      __LINE__, __FUNCTION__, __FILE__);
        }
        catch (const std::exception& e)
        {
            error(e.what(), __LINE__, __FUNCTION__, __FILE__);
        }
    }

    template<typename T>
    ArrayCpuGpu<T>::ArrayCpuGpu(const int num, const int channels, const int height, const int width)
        : spImpl{std::make_shared<ImplArrayCpuGpu>()}
    {
        spImpl->reshape({num, channels, height, width});
    }

    template<typename T>
    void ArrayCpuGpu<T>::Reshape(const int num, const int channels, const int height, const int width)
    {
        spImpl->reshape({num, channels, height, width});
    }

    template<typename T>
    void ArrayCpuGpu<T>::Reshape(const std::vector<int>& shape)
    {
        spImpl->reshape(shape);
    }

    template<typename T>
    std::string ArrayCpuGpu<T>::shape_string() const
    {
        std::ostringstream stream;
        for (const auto d : spImpl->shape)
            stream << d << " ";
        stream << "(" << spImpl->count << ")";
        return stream.str();
    }

    template<typename T>
    const std::vector<int>& ArrayCpuGpu<T>::shape() const
    {
        return spImpl->shape;
    }

    template<typename T>
    int ArrayCpuGpu<T>::shape(const int index) const
    {
        return spImpl->shape[CanonicalAxisIndex(index)];
    }

    template<typename T>
    int ArrayCpuGpu<T>::num_axes() const
    {
        return (int)spImpl->shape.size();
    }

    template<typename T>
    int ArrayCpuGpu<T>::count() const
    {
        return spImpl->count;
    }

    template<typename T>
    int ArrayCpuGpu<T>::count(const int start_axis, const int end_axis) const
    {
        if (start_axis > end_axis || start_axis < 0 || end_axis < 0 || start_axis > num_axes() ||
            end_axis > num_axes())
            error("count: bad axis range.", __LINE__, __FUNCTION__, __FILE__);
        int c = 1;
        for (int i = start_axis; i < end_axis; ++i)
            c *= spImpl->shape[i];
        return c;
    }

    template<typename T>
    int ArrayCpuGpu<T>::count(const int start_axis) const
    {
        return count(start_axis, num_axes());
    }

    template<typename T>
    int ArrayCpuGpu<T>::CanonicalAxisIndex(const int axis_index) const
    {
        if (axis_index < -num_axes() || axis_index >= num_axes())
            error("axis " + std::to_string(axis_index) + " out of range for a " +
                  std::to_string(num_axes()) + "-D blob.", __LINE__, __FUNCTION__, __FILE__);
        return axis_index < 0 ? axis_index + num_axes() : axis_index;
    }

    template<typename T>
    int ArrayCpuGpu<T>::num() const { return LegacyShape(0); }
    template<typename T>
    int ArrayCpuGpu<T>::channels() const { return LegacyShape(1); }
    template<typename T>
    int ArrayCpuGpu<T>::height() const { return LegacyShape(2); }
    template<typename T>
    int ArrayCpuGpu<T>::width() const { return LegacyShape(3); }

    template<typename T>
    int ArrayCpuGpu<T>::LegacyShape(const int index) const
    {
        if (num_axes() > 4)
            error("Cannot use legacy accessors on Blobs with > 4 axes.", __LINE__, __FUNCTION__, __FILE__);
        if (index >= num_axes() || index < -num_axes())
            return 1;
        return shape(index);
    }

    template<typename T>
    int ArrayCpuGpu<T>::offset(const int n, const int c, const int h, const int w) const
    {
        return ((n * channels() + c) * height() + h) * width() + w;
    }

    template<typename T>
    T ArrayCpuGpu<T>::data_at(const int n, const int c, const int h, const int w) const
    {
        return cpu_data()[offset(n, c, h, w)];
    }

    template<typename T>
    T ArrayCpuGpu<T>::diff_at(const int n, const int c, const int h, const int w) const
    {
        return cpu_diff()[offset(n, c, h, w)];
    }

    template<typename T>
    const T* ArrayCpuGpu<T>::cpu_data() const
    {
        return spImpl->data ? static_cast<const T*>(spImpl->data->cpu()) : nullptr;
    }

    template<typename T>
    void ArrayCpuGpu<T>::set_cpu_data(T* data)
    {
        if (!spImpl->data)
            error("set_cpu_data on an unshaped blob.", __LINE__, __FUNCTION__, __FILE__);
        spImpl->data->setCpu(data, (size_t)spImpl->count * sizeof(T));
    }

    template<typename T>
    const int* ArrayCpuGpu<T>::gpu_shape() const
    {
        return spImpl->shapeData ? static_cast<const int*>(spImpl->shapeData->gpu()) : nullptr;
    }

    template<typename T>
    const T* ArrayCpuGpu<T>::gpu_data() const
    {
        return spImpl->data ? static_cast<const T*>(spImpl->data->gpu()) : nullptr;
    }

    template<typename T>
    void ArrayCpuGpu<T>::set_gpu_data(T* data)
    {
        if (!spImpl->data)
            error("set_gpu_data on an unshaped blob.", __LINE__, __FUNCTION__, __FILE__);
        spImpl->data->setGpu(data, (size_t)spImpl->count * sizeof(T));
    }

    template<typename T>
    const T* ArrayCpuGpu<T>::cpu_diff() const
    {
        return spImpl->diff ? static_cast<const T*>(spImpl->diff->cpu()) : nullptr;
    }

    template<typename T>
    const T* ArrayCpuGpu<T>::gpu_diff() const
    {
        return spImpl->diff ? static_cast<const T*>(spImpl->diff->gpu()) : nullptr;
    }

    template<typename T>
    T* ArrayCpuGpu<T>::mutable_cpu_data()
    {
        return spImpl->data ? static_cast<T*>(spImpl->data->mutableCpu()) : nullptr;
    }

    template<typename T>
    T* ArrayCpuGpu<T>::mutable_gpu_data()
    {
        return spImpl->data ? static_cast<T*>(spImpl->data->mutableGpu()) : nullptr;
    }

    template<typename T>
    T* ArrayCpuGpu<T>::mutable_cpu_diff()
    {
        return spImpl->diff ? static_cast<T*>(spImpl->diff->mutableCpu()) : nullptr;
    }

    template<typename T>
    T* ArrayCpuGpu<T>::mutable_gpu_diff()
    {
        return spImpl->diff ? static_cast<T*>(spImpl->diff->mutableGpu()) : nullptr;
    }

    template<typename T>
    void ArrayCpuGpu<T>::Update()
    {
        // Blob::Update: data -= diff
        if (!spImpl->data)
            return;
        const T* d = cpu_diff();
        T* x = mutable_cpu_data();
        for (int i = 0; i < count(); ++i)
            x[i] = T(x[i] - d[i]);
    }

    template<typename T>
    T ArrayCpuGpu<T>::asum_data() const
    {
        T s = T(0);
        const T* x = cpu_data();
        for (int i = 0; i < count(); ++i)
            s += T(x[i] < T(0) ? -x[i] : x[i]);
        return s;
    }

    template<typename T>
    T ArrayCpuGpu<T>::asum_diff() const
    {
        T s = T(0);
        const T* x = cpu_diff();
        for (int i = 0; i < count(); ++i)
            s += T(x[i] < T(0) ? -x[i] : x[i]);
        return s;
    }

    template<typename T>
    T ArrayCpuGpu<T>::sumsq_data() const
    {
        T s = T(0);
        const T* x = cpu_data();
        for (int i = 0; i < count(); ++i)
            s += T(x[i] * x[i]);
        return s;
    }

    template<typename T>
    T ArrayCpuGpu<T>::sumsq_diff() const
    {
        T s = T(0);
        const T* x = cpu_diff();
        for (int i = 0; i < count(); ++i)
            s += T(x[i] * x[i]);
        return s;
    }

    template<typename T>
    void ArrayCpuGpu<T>::scale_data(const T scale_factor)
    {
        T* x = mutable_cpu_data();
        for (int i = 0; i < count(); ++i)
            x[i] = T(x[i] * scale_factor);
    }

    template<typename T>
    void ArrayCpuGpu<T>::scale_diff(const T scale_factor)
    {
        T* x = mutable_cpu_diff();
        for (int i = 0; i < count(); ++i)
            x[i] = T(x[i] * scale_factor);
    }

    COMPILE_TEMPLATE_FLOATING_INT_TYPES_CLASS(ArrayCpuGpu);
}
