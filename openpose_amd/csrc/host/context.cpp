// context.cpp -- cached device tables of a context.
#include "context.h"

#include <cmath>

namespace opk {

// OpenCV's generic INTER_CUBIC setup (cv::resize, imgproc/src/resize.cpp, the third-party code
// behind resizeAndMergeBase.cpp:51): scale = 1/((double)d/s); f = (float)((i+0.5)*scale-0.5);
// s0 = floor(f); t = f - s0; Keys coefficients with A = -0.75 in float.  Built with
// -ffp-contract=off so the coefficients equal the CPU path's bit for bit.
void cubic_tables(int s, int d, int* ofs, float* coef)
{
    const double scale = 1. / ((double)d / s);
    const float A = -0.75f;
    for (int i = 0; i < d; ++i) {
        float f = (float)((i + 0.5) * scale - 0.5);
        const int s0 = (int)std::floor(f);
        f -= (float)s0;
        ofs[i] = s0;
        float* c = coef + 4 * i;
        c[0] = ((A * (f + 1) - 5 * A) * (f + 1) + 8 * A) * (f + 1) - 4 * A;
        c[1] = ((A + 2) * f - (A + 3)) * f * f + 1;
        c[2] = ((A + 2) * (1 - f) - (A + 3)) * (1 - f) * (1 - f) + 1;
        c[3] = 1.f - c[0] - c[1] - c[2];
    }
}

const Context::Tables& Context::tables(int sh, int sw, int dh, int dw)
{
    auto key = std::make_tuple(sh, sw, dh, dw);
    auto it = resize_tables.find(key);
    if (it != resize_tables.end()) return *it->second;
    auto t = std::make_unique<Tables>();
    // layout: ycoef [dh][4] | xcoef [dw][4] | yofs [dh] | xofs [dw]  (float4-aligned coefs first)
    std::vector<char> host((size_t)(dh + dw) * 20);
    float* yc = reinterpret_cast<float*>(host.data());
    float* xc = yc + 4 * dh;
    int* yo = reinterpret_cast<int*>(xc + 4 * dw);
    int* xo = yo + dh;
    cubic_tables(sh, dh, yo, yc);
    cubic_tables(sw, dw, xo, xc);
    char* dev = static_cast<char*>(t->buf.get(host.size()));
    OPK_HIP(hipMemcpyAsync(dev, host.data(), host.size(), hipMemcpyHostToDevice, stream));
    OPK_HIP(hipStreamSynchronize(stream));   // `host` dies at return
    t->ycoef = reinterpret_cast<const float*>(dev);
    t->xcoef = t->ycoef + 4 * dh;
    t->yofs = reinterpret_cast<const int*>(t->xcoef + 4 * dw);
    t->xofs = t->yofs + dh;
    auto& ref = *t;
    resize_tables.emplace(key, std::move(t));
    return ref;
}

const PafPairTable& Context::pose_table(int model)
{
    auto it = pose_dev.find(model);
    if (it != pose_dev.end()) return it->second->t;
    const PoseModelInfo& m = pose_model(model);
    const int np = m.npairs();
    std::vector<int> host(4 * np);
    const int base = m.parts + (m.bkg ? 1 : 0);
    for (int q = 0; q < np; ++q) {
        host[2 * q] = m.pairs[2 * q];
        host[2 * q + 1] = m.pairs[2 * q + 1];
        host[2 * np + q] = base + m.map_idx[2 * q];
        host[3 * np + q] = base + m.map_idx[2 * q + 1];
    }
    auto d = std::make_unique<PoseDev>();
    int* dev = static_cast<int*>(d->buf.get(host.size() * sizeof(int)));
    OPK_HIP(hipMemcpyAsync(dev, host.data(), host.size() * sizeof(int), hipMemcpyHostToDevice,
                           stream));
    OPK_HIP(hipStreamSynchronize(stream));
    d->t = PafPairTable{np, m.parts, dev, dev + 2 * np, dev + 3 * np};
    auto& ref = d->t;
    pose_dev.emplace(model, std::move(d));
    return ref;
}

int* Context::nms_candidates(int frames, int parts)
{
    const size_t need = nms_scratch_ints(frames, parts) * sizeof(int);
    if (need > nms_scratch.bytes) {
        nms_scratch.get(need);
        OPK_HIP(hipMemsetAsync(nms_scratch.ptr, 0, need, stream));
    }
    return static_cast<int*>(nms_scratch.ptr);
}

EventTimer::~EventTimer()
{
    for (auto* v : {&events_, &free_})
        for (auto& e : *v) {
            (void)hipEventDestroy(e.first);
            (void)hipEventDestroy(e.second);
        }
}

void EventTimer::begin(hipStream_t s)
{
    if (!on) return;
    if (free_.empty()) {
        std::pair<hipEvent_t, hipEvent_t> e;
        OPK_HIP(hipEventCreate(&e.first));
        OPK_HIP(hipEventCreate(&e.second));
        free_.push_back(e);
    }
    events_.push_back(free_.back());
    free_.pop_back();
    OPK_HIP(hipEventRecord(events_.back().first, s));
}

void EventTimer::end(hipStream_t s)
{
    if (on && !events_.empty()) OPK_HIP(hipEventRecord(events_.back().second, s));
}

void EventTimer::read(int* count, double* total_ms)
{
    double t = 0;
    for (auto& e : events_) {
        OPK_HIP(hipEventSynchronize(e.second));
        float ms = 0.f;
        OPK_HIP(hipEventElapsedTime(&ms, e.first, e.second));
        t += ms;
        free_.push_back(e);
    }
    if (count) *count = (int)events_.size();
    if (total_ms) *total_ms = t;
    events_.clear();
}

}  // namespace opk
