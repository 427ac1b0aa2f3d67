// connector.h -- host people assembly of the body-part connector (product code).
#pragma once
#include <vector>

#include "pose_model.h"

namespace opk {

// Where the PAF score of (pair q, 1-based peak i of A, 1-based peak j of B) is read from.
struct PairScores {
    const float* data = nullptr;
    int max_peaks = 0;     // dense layout [npairs][max_peaks][max_peaks]
    bool compact = false;  // compact layout: pair blocks of nA*nB, offsets[q]
    const int* offsets = nullptr;
    float at(int q, int i, int j, int nb) const
    {
        if (compact) return data[offsets[q] + (i - 1) * nb + (j - 1)];
        return data[((size_t)q * max_peaks + (i - 1)) * max_peaks + (j - 1)];
    }
};

constexpr int kConnectCpu = 0;   // connectBodyPartsCpu assembly (BODY_25 / COCO / MPI)
constexpr int kConnectGpu = 1;   // connectBodyPartsGpu assembly (every model, BODY_135 included)

struct ConnectParams {
    int min_subset_cnt = 3;
    float min_subset_score = 0.4f;
    float scale = 1.f;
    bool maximize_positives = false;
    int semantics = kConnectCpu;
};

// People assembly from precomputed pair scores with the connectBodyPartsCpu
// (bodyPartConnectorBase.cpp:1327-1377) or connectBodyPartsGpu (bodyPartConnectorBase.cu:147-250)
// semantics.  peaks: [parts][max_peaks+1][3] host.  Fills kp [P][parts][3] and ks [P]; returns P.
int assemble_people(const PoseModelInfo& model, const float* peaks, int max_peaks,
                    const PairScores& scores, const ConnectParams& p, std::vector<float>& kp,
                    std::vector<float>& ks);

// compact-score offsets of every pair for the given peaks (returns the total count)
int compact_offsets(const PoseModelInfo& model, const float* peaks, int max_peaks,
                    std::vector<int>& offsets);

}  // namespace opk
