// connector.h -- host people assembly of the body-part connector (product code).
#pragma once
#include <cstddef>
#include <cstdint>
#include <vector>

#include "pose_model.h"

namespace opk {

// Where the PAF score of (pair q, 1-based peak i of A, 1-based peak j of B) is read from.
struct PairScores {
    const float* data = nullptr;
    int max_peaks = 0;     // dense layout [npairs][max_peaks][max_peaks]
    bool compact = false;  // compact layout: pair blocks of nA*nB, offsets[q]
    const int* offsets = nullptr;
    float at(int q, int i, int j, int nb) const { return row(q, i, nb)[j - 1]; }
    const float* row(int q, int i, int nb) const   // the scores of A peak i against B peaks 1..nb
    {
        if (compact) return data + offsets[q] + (size_t)(i - 1) * nb;
        return data + ((size_t)q * max_peaks + (i - 1)) * max_peaks;
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

// Working storage of one assembly, reusable across frames (a worker thread keeps one, so a batch's
// frames allocate nothing once the buffers have grown to the largest frame seen)
struct AssemblyScratch {
    struct Key {        // one connection, ordered as the reference's std::greater on
        uint64_t hi;    // (total, paf, pair, peak A, peak B): hi = (total, paf) as ordered bits,
        uint64_t lo;    // lo = pair << 32 | i << 16 | j
    };
    std::vector<Key> keys, keys_tmp;
    std::vector<int> slot, found, owner, node_part, node_next, head, tail, dead, keep;
    std::vector<float> score;
};

// People assembly from precomputed pair scores with the connectBodyPartsCpu
// (bodyPartConnectorBase.cpp:1327-1377) or connectBodyPartsGpu (bodyPartConnectorBase.cu:147-250)
// semantics.  peaks: [parts][max_peaks+1][3] host.  Fills kp [P][parts][3] and ks [P]; returns P.
int assemble_people(const PoseModelInfo& model, const float* peaks, int max_peaks,
                    const PairScores& scores, const ConnectParams& p, std::vector<float>& kp,
                    std::vector<float>& ks, AssemblyScratch* scratch = nullptr);

// compact-score offsets of every pair for the given peaks (returns the total count)
int compact_offsets(const PoseModelInfo& model, const float* peaks, int max_peaks,
                    std::vector<int>& offsets);

}  // namespace opk
