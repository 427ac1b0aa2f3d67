// render_driver.cpp -- test driver for integration/renderHip.cpp: calls the reference's render entry
// points (include/openpose/pose/renderPose.hpp, face/renderFace.hpp) with their own signatures.
//
// Built against the reference headers by tests/test_render_shim.py.  `render_driver DIR` reads
// DIR/meta.i32 {w, h, people, hw, hh, faces}, DIR/frame.f32 [h][w][3], DIR/pose.f32 [people][25][3],
// DIR/heat.f32 [78][hh][hw], DIR/face.f32 [faces][70][3] and writes DIR/out_pose.f32,
// out_heat.f32, out_pafs.f32, out_face.f32 (each render on a fresh copy of the frame); then checks
// that an invalid call comes back through op::error.
#include <cstdio>
#include <stdexcept>
#include <string>
#include <vector>

#include <openpose/face/renderFace.hpp>
#include <openpose/pose/renderPose.hpp>
#include <openpose/utilities/errorAndLog.hpp>

#include "opk.h"
#include "opk_shim.hpp"

namespace op
{
    void error(const std::string& message, const int line, const std::string& function,
               const std::string& file)
    {
        throw std::runtime_error(message + " (" + file + ":" + std::to_string(line) + " " + function + ")");
    }

    OpkContext opkShimThreadContext(const int)
    {
        static OpkContext ctx;
        if (!ctx) {
            opk_ctx* raw = nullptr;
            if (opk_ctx_create(0, nullptr, &raw) != OPK_OK)
                throw std::runtime_error(opk_last_error());
            ctx = OpkContext{raw, opk_ctx_destroy};
        }
        return ctx;
    }
}

namespace
{
    template <typename T>
    std::vector<T> load(const std::string& path, size_t n)
    {
        std::vector<T> v(n);
        FILE* f = std::fopen(path.c_str(), "rb");
        if (!f || std::fread(v.data(), sizeof(T), n, f) != n)
            throw std::runtime_error("cannot read " + path);
        std::fclose(f);
        return v;
    }

    void save(const std::string& path, const std::vector<float>& v)
    {
        FILE* f = std::fopen(path.c_str(), "wb");
        if (!f || std::fwrite(v.data(), sizeof(float), v.size(), f) != v.size())
            throw std::runtime_error("cannot write " + path);
        std::fclose(f);
    }

    void* upload(const void* host, size_t bytes)
    {
        void* dev = nullptr;
        if (opk_malloc(op::opkShimThreadContext().get(), &dev, bytes ? bytes : 4) != OPK_OK ||
            opk_memcpy_h2d(op::opkShimThreadContext().get(), dev, host, bytes) != OPK_OK)
            throw std::runtime_error(opk_last_error());
        return dev;
    }
}

int main(int argc, char** argv)
{
    try {
        if (argc < 2) throw std::runtime_error("usage: render_driver DIR");
        const std::string dir = argv[1];
        const auto meta = load<int>(dir + "/meta.i32", 6);
        const int w = meta[0], h = meta[1], people = meta[2], hw = meta[3], hh = meta[4], faces = meta[5];
        const size_t fn = (size_t)w * h * 3;
        const auto frame = load<float>(dir + "/frame.f32", fn);
        const auto pose = load<float>(dir + "/pose.f32", (size_t)people * 25 * 3);
        const auto heat = load<float>(dir + "/heat.f32", (size_t)78 * hw * hh);
        const auto face = load<float>(dir + "/face.f32", (size_t)faces * 70 * 3);
        opk_ctx* ctx = op::opkShimThreadContext().get();
        float* dframe = static_cast<float*>(upload(frame.data(), fn * 4));
        const float* dpose = static_cast<const float*>(upload(pose.data(), pose.size() * 4));
        const float* dheat = static_cast<const float*>(upload(heat.data(), heat.size() * 4));
        const float* dface = static_cast<const float*>(upload(face.data(), face.size() * 4));
        // op::Point's members live in the reference's core/point.cpp, which this driver does not
        // build (no reference code travels to the GPU box): the two plain fields are laid out as the
        // class declares them (point.hpp:12-13) and only read through the const references
        const unsigned size_raw[2] = {(unsigned)w, (unsigned)h};
        const int hsize_raw[2] = {hw, hh};
        const auto& size = *reinterpret_cast<const op::Point<unsigned int>*>(size_raw);
        const auto& hsize = *reinterpret_cast<const op::Point<int>*>(hsize_raw);
        const float scale = (float)w / (float)hw;
        std::vector<float> out(fn);
        auto fetch = [&](const char* name) {
            if (opk_memcpy_d2h(ctx, out.data(), dframe, fn * 4) != OPK_OK)
                throw std::runtime_error(opk_last_error());
            save(dir + "/" + name, out);
            if (opk_memcpy_h2d(ctx, dframe, frame.data(), fn * 4) != OPK_OK)
                throw std::runtime_error(opk_last_error());
        };
        op::renderPoseKeypointsGpu(dframe, nullptr, nullptr, nullptr, op::PoseModel::BODY_25, people,
                                   size, dpose, 0.05f, true, true, 0.6f);
        fetch("out_pose.f32");
        op::renderPoseHeatMapGpu(dframe, size, dheat, hsize, scale, 3u, 0.7f);
        fetch("out_heat.f32");
        op::renderPosePAFsGpu(dframe, op::PoseModel::BODY_25, size, dheat, hsize, scale, 0.7f);
        fetch("out_pafs.f32");
        op::renderFaceKeypointsGpu(dframe, nullptr, nullptr, nullptr, size, dface, faces, 0.4f, 0.6f);
        fetch("out_face.f32");
        bool threw = false;
        try {
            op::renderPoseKeypointsGpu(dframe, nullptr, nullptr, nullptr, op::PoseModel::MPI_15, 1,
                                       size, dpose, 0.05f, true, true, 0.6f);
        } catch (const std::exception& e) {
            threw = std::string(e.what()).find("googlyEyes") != std::string::npos;
        }
        if (!threw) throw std::runtime_error("MPI + googly eyes did not error");
        std::printf("render ok\n");
        return 0;
    } catch (const std::exception& e) {
        std::fprintf(stderr, "exception: %s\n", e.what());
        return 1;
    }
}
