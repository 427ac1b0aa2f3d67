// connector.cpp -- host people assembly (product code, runs on the GPU worker's host thread).
//
// Semantics of the reference CPU path, /root/reference/src/openpose/net/bodyPartConnectorBase.cpp:
//   createPeopleVector (:156-472) fed by precomputed pair scores (its :321-340 input),
//   removePeopleBelowThresholdsAndFillFaces (:720-884) for <= 65-part models,
//   peopleVectorToPeopleArray (:886-934).
// The PAF line integrals come from the GPU (kernels/paf.hip); this file only sorts, matches and
// groups.  People are stored flat (one int row of `parts` score indices per person) instead of a
// vector of vectors; the arithmetic on scores follows the reference operation for operation
// (double-promoted sums where the reference's tuple holds a double).
#include "connector.h"

#include <algorithm>
#include <cmath>

namespace opk {

namespace {

inline int round_pos(float a) { return int(a + 0.5f); }

struct Cand {
    double s;
    int i, j;
};
inline bool cand_greater(const Cand& a, const Cand& b)
{
    if (a.s != b.s) return a.s > b.s;
    if (a.i != b.i) return a.i > b.i;
    return a.j > b.j;
}

struct People {
    int parts;
    std::vector<int> slot;     // [n][parts]
    std::vector<int> found;    // parts counter of each person
    std::vector<float> score;  // running score
    int size() const { return (int)found.size(); }
    int* row(int p) { return slot.data() + (size_t)p * parts; }
    const int* row(int p) const { return slot.data() + (size_t)p * parts; }
    int add()
    {
        slot.resize(slot.size() + parts, 0);
        found.push_back(0);
        score.push_back(0.f);
        return size() - 1;
    }
};

}  // namespace

int compact_offsets(const PoseModelInfo& m, const float* peaks, int max_peaks,
                    std::vector<int>& offsets)
{
    const int stride = 3 * (max_peaks + 1);
    offsets.resize(m.npairs());
    int off = 0;
    for (int q = 0; q < m.npairs(); ++q) {
        offsets[q] = off;
        off += round_pos(peaks[m.pairs[2 * q] * stride]) * round_pos(peaks[m.pairs[2 * q + 1] * stride]);
    }
    return off;
}

int assemble_people(const PoseModelInfo& m, const float* peaks, int max_peaks,
                    const PairScores& scores, const ConnectParams& prm, std::vector<float>& kp,
                    std::vector<float>& ks)
{
    const int P = m.parts;
    const int stride = 3 * (max_peaks + 1);
    People people{P, {}, {}, {}};
    std::vector<Cand> cand;
    std::vector<int> chosenA, chosenB;
    std::vector<double> chosenS;
    std::vector<char> usedA, usedB;

    for (int q = 0; q < m.npairs(); ++q) {
        const int pa = m.pairs[2 * q], pb = m.pairs[2 * q + 1];
        const int na = round_pos(peaks[pa * stride]);
        const int nb = round_pos(peaks[pb * stride]);
        if (na == 0 || nb == 0) {
            // one side has no candidates: the other side's peaks become 1-part people
            // (deduplicated, except for the 15-part MPI models)
            const int part = na == 0 ? pb : pa;
            const int cnt = na == 0 ? nb : na;
            for (int i = 1; i <= cnt; ++i) {
                const int s = part * stride + i * 3 + 2;
                bool dup = false;
                if (P != 15)
                    for (int p = 0; p < people.size() && !dup; ++p) dup = people.row(p)[part] == s;
                if (dup) continue;
                const int p = people.add();
                people.row(p)[part] = s;
                people.found[p] = 1;
                people.score[p] = peaks[s];
            }
            continue;
        }
        cand.clear();
        for (int i = 1; i <= na; ++i)
            for (int j = 1; j <= nb; ++j) {
                const float s = scores.at(q, i, j, nb);
                if (s > 1e-6) cand.push_back({(double)s, i, j});
            }
        std::sort(cand.begin(), cand.end(), cand_greater);
        chosenA.clear(); chosenB.clear(); chosenS.clear();
        usedA.assign(na, 0);
        usedB.assign(nb, 0);
        const int limit = std::min(na, nb);
        for (const Cand& c : cand) {
            if (usedA[c.i - 1] || usedB[c.j - 1]) continue;
            chosenA.push_back(pa * stride + c.i * 3 + 2);
            chosenB.push_back(pb * stride + c.j * 3 + 2);
            chosenS.push_back(c.s);
            if ((int)chosenA.size() == limit) break;
            usedA[c.i - 1] = 1;
            usedB[c.j - 1] = 1;
        }
        const int nc = (int)chosenA.size();
        if (nc == 0) continue;
        const bool ear = (P == 18 && (q == 17 || q == 18)) ||
                         ((P == 19 || P == 25 || P == 59 || P == 65) && (q == 18 || q == 19));
        if (q == 0) {
            for (int c = 0; c < nc; ++c) {
                const int p = people.add();
                people.row(p)[m.pairs[0]] = chosenA[c];
                people.row(p)[m.pairs[1]] = chosenB[c];
                people.found[p] = 2;
                people.score[p] = float(peaks[chosenA[c]] + peaks[chosenB[c]] + chosenS[c]);
            }
        } else if (ear) {
            for (int c = 0; c < nc; ++c)
                for (int p = 0; p < people.size(); ++p) {
                    int* r = people.row(p);
                    if (r[pa] == chosenA[c] && r[pb] == 0) r[pb] = chosenB[c];
                    else if (r[pb] == chosenB[c] && r[pa] == 0) r[pa] = chosenA[c];
                }
        } else {
            for (int c = 0; c < nc; ++c) {
                int hit = -1;
                for (int p = 0; p < people.size(); ++p)
                    if (people.row(p)[pa] == chosenA[c]) { hit = p; break; }
                if (hit >= 0) {
                    people.row(hit)[pb] = chosenB[c];
                    people.found[hit]++;
                    people.score[hit] += peaks[chosenB[c]] + float(chosenS[c]);
                } else {
                    const int p = people.add();
                    people.row(p)[pa] = chosenA[c];
                    people.row(p)[pb] = chosenB[c];
                    people.found[p] = 2;
                    people.score[p] = float(peaks[chosenA[c]] + peaks[chosenB[c]] + chosenS[c]);
                }
            }
        }
    }

    // thresholds (removePeopleBelowThresholdsAndFillFaces, <= 65-part models), with the
    // second pass at maximizePositives = true when nobody survives
    std::vector<int> keep;
    auto select = [&](bool maxpos) {
        keep.clear();
        for (int p = 0; p < people.size(); ++p) {
            int counter = people.found[p];
            if (!maxpos && (P == 25 || P > 70)) {
                int foot = 0;
                for (int k = 19; k < 25; ++k) foot += people.row(p)[k] > 0;
                if (foot > 0) {
                    counter -= foot;
                    if (counter <= 4) continue;
                }
            }
            if (counter >= prm.min_subset_cnt && (people.score[p] / counter) >= prm.min_subset_score)
                keep.push_back(p);
        }
    };
    select(prm.maximize_positives);
    if (keep.empty() && !prm.maximize_positives) select(true);

    const int n = (int)keep.size();
    kp.assign((size_t)n * P * 3, 0.f);
    ks.assign(n, 0.f);
    const float inv = 1 / float(P + m.npairs());
    for (int o = 0; o < n; ++o) {
        const int* r = people.row(keep[o]);
        float* d = kp.data() + (size_t)o * P * 3;
        for (int k = 0; k < P; ++k) {
            const int s = r[k];
            if (s > 0) {
                d[3 * k] = peaks[s - 2] * prm.scale;
                d[3 * k + 1] = peaks[s - 1] * prm.scale;
                d[3 * k + 2] = peaks[s];
            }
        }
        ks[o] = people.score[keep[o]] * inv;
    }
    return n;
}

}  // namespace opk
