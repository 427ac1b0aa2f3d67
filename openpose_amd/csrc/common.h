// common.h -- internal helpers shared by the HIP kernels and the C++ host of libopk_hip.so.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>
#include <stdexcept>
#include <string>
#include <vector>

namespace opk {

// Thread-local error message behind opk_last_error() (C-ABI error convention, include/opk.h).
void set_error(const std::string& msg);

struct Error : std::runtime_error {
    int code;
    Error(int c, const std::string& m) : std::runtime_error(m), code(c) {}
};

#define OPK_CHECK_ARG(cond, msg)                                                              \
    do {                                                                                      \
        if (!(cond)) throw ::opk::Error(1, std::string(__func__) + ": " + (msg));             \
    } while (0)

#define OPK_HIP(call)                                                                         \
    do {                                                                                      \
        hipError_t e_ = (call);                                                               \
        if (e_ != hipSuccess)                                                                 \
            throw ::opk::Error(2, std::string(#call) + " failed: " + hipGetErrorString(e_) +   \
                                      " (" + __FILE__ + ":" + std::to_string(__LINE__) + ")");  \
    } while (0)

// after a kernel launch (reference: cudaCheck -> cudaPeekAtLastError, gpu/cuda.cpp:18-26)
#define OPK_LAUNCH_CHECK() OPK_HIP(hipPeekAtLastError())

// Kernel-variant switches (A/B tests and tuning only): a process-wide table written solely through
// opk_dev_set (include/opk.h) -- never read from the environment, so nothing a user's shell
// exports can change which kernels run.  Unset keys give dflt (the product configuration).
int dev_switch(const char* key, int dflt);

// Launch log (tests and profiling: which kernel instantiation ran for which layer).  While a
// log is attached to the calling thread, note_launch() appends "<layer>\t<kernel>" lines to it;
// otherwise it returns at once.  NetHip attaches its log for the forwards run while the dev
// switch LAUNCH_LOG is 1 (opk_net_launch_log).
struct LaunchLog {
    std::string layer;
    std::vector<std::string> lines;
};
void attach_launch_log(LaunchLog* log);   // nullptr detaches
LaunchLog* launch_log();
void note_launch(const char* fmt, ...) __attribute__((format(printf, 1, 2)));

// Device scratch that only grows (one per context and purpose); never freed inside a launch
// sequence so the launch functions stay graph-capturable.
struct DevBuf {
    void* ptr = nullptr;
    size_t bytes = 0;
    void* get(size_t need) {
        if (need > bytes) {
            if (ptr) OPK_HIP(hipFree(ptr));
            ptr = nullptr;
            OPK_HIP(hipMalloc(&ptr, need));
            bytes = need;
        }
        return ptr;
    }
    ~DevBuf() { if (ptr) (void)hipFree(ptr); }
};

struct HostBuf {   // pinned host staging
    void* ptr = nullptr;
    size_t bytes = 0;
    void* get(size_t need) {
        if (need > bytes) {
            if (ptr) OPK_HIP(hipHostFree(ptr));
            ptr = nullptr;
            OPK_HIP(hipHostMalloc(&ptr, need, hipHostMallocDefault));
            bytes = need;
        }
        return ptr;
    }
    ~HostBuf() { if (ptr) (void)hipHostFree(ptr); }
};

}  // namespace opk
