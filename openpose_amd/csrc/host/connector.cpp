// connector.cpp -- host people assembly (product code, runs on the GPU worker's host thread).
//
// Two assembly semantics of /root/reference/src/openpose/net/bodyPartConnectorBase.cpp:
//   CPU path (connectBodyPartsCpu :1327-1377, BODY_25 / COCO / MPI only): createPeopleVector
//     (:156-472) fed by precomputed pair scores (its :321-340 input);
//   GPU path (connectBodyPartsGpu, bodyPartConnectorBase.cu:147-250, every model incl. BODY_135):
//     pafPtrIntoVector (:474-541, one global sort of all connections) + pafVectorIntoPeopleVector
//     (:543-718, create / extend / merge people);
// then, for both, removePeopleBelowThresholdsAndFillFaces (:720-884, with the >= 135-part hand and
// face counting and the face-fragment merge via getKeypointsRoi, utilities/keypoint.cpp:586-632)
// and peopleVectorToPeopleArray (:886-934).
// The PAF line integrals come from the GPU (kernels/paf.hip); this file only sorts, matches and
// groups.  People are stored flat (one int row of `parts` score indices per person) instead of a
// vector of vectors; the arithmetic on scores follows the reference operation for operation
// (double-promoted sums where the reference's tuple holds a double).
#include "connector.h"

#include <algorithm>
#include <cmath>
#include <cstring>
#if defined(__SSE__)
#include <immintrin.h>
#endif
#include <limits>
#include <string>

#include "../common.h"

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

struct People {   // rows live in an AssemblyScratch (cleared, capacity kept)
    int parts;
    std::vector<int>& slot;     // [n][parts]
    std::vector<int>& found;    // parts counter of each person
    std::vector<float>& score;  // running score
    People(int P, AssemblyScratch& s) : parts(P), slot(s.slot), found(s.found), score(s.score)
    {
        slot.clear();
        found.clear();
        score.clear();
    }
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

// the smallest float above the reference's 1e-6 PAF-score cut (a double literal)
const float kPafMinFloat = (double)(float)1e-6 > 1e-6 ? (float)1e-6
                                                       : std::nextafter((float)1e-6, 1.f);

// float <-> unsigned with the same order (non-NaN; -0 never occurs: every connection total and
// PAF score is a sum with a positive PAF term)
inline uint32_t ordered_bits(float f)
{
    uint32_t u;
    std::memcpy(&u, &f, 4);
    return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}
inline float from_ordered_bits(uint32_t u)
{
    u = (u & 0x80000000u) ? (u & 0x7fffffffu) : ~u;
    float f;
    std::memcpy(&f, &u, 4);
    return f;
}

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

namespace {

// createPeopleVector (CPU path): pair by pair, greedy one-to-one matching per pair
void people_per_pair(People& people, const PoseModelInfo& m, const float* peaks, int max_peaks,
                     const PairScores& scores)
{
    const int P = m.parts;
    const int stride = 3 * (max_peaks + 1);
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

}

// Keys -> descending (hi, lo): an LSD radix sort of ~total (hi's upper 32 bits; 3 passes of 11
// bits, a pass skipped when every key has the same digit), then every run of equal totals
// (rare: two connections with bit-identical float sums) ordered by (paf, lo) descending in place.
// A BODY_135 frame of 20 people holds ~3000 connections: 3-4x faster than a comparison sort, and
// half the passes of a radix sort over all 64 bits of hi.
void sort_descending(std::vector<AssemblyScratch::Key>& keys, std::vector<AssemblyScratch::Key>& tmp)
{
    const size_t n = keys.size();
    auto greater = [](const AssemblyScratch::Key& a, const AssemblyScratch::Key& b) {
        return a.hi != b.hi ? a.hi > b.hi : a.lo > b.lo;
    };
    if (n < 64) {
        std::sort(keys.begin(), keys.end(), greater);
        return;
    }
    constexpr int kBits = 11, kPasses = 3, kBuckets = 1 << kBits;
    uint32_t hist[kPasses][kBuckets] = {};
    auto digit = [](uint64_t hi, int d) { return (uint32_t)((~hi >> (32 + kBits * d)) & (kBuckets - 1)); };
    for (const auto& k : keys)
        for (int d = 0; d < kPasses; ++d) ++hist[d][digit(k.hi, d)];
    tmp.resize(n);
    AssemblyScratch::Key* src = keys.data();
    AssemblyScratch::Key* dst = tmp.data();
    for (int d = 0; d < kPasses; ++d) {
        uint32_t* h = hist[d];
        if (h[digit(src[0].hi, d)] == n) continue;   // one digit value
        uint32_t sum = 0;
        for (int b = 0; b < kBuckets; ++b) {
            const uint32_t c = h[b];
            h[b] = sum;
            sum += c;
        }
        for (size_t i = 0; i < n; ++i) dst[h[digit(src[i].hi, d)]++] = src[i];
        std::swap(src, dst);
    }
    if (src != keys.data()) std::copy(src, src + n, keys.data());
    // equal totals: (paf, lo) descending
    for (size_t i = 0; i + 1 < n;) {
        size_t j = i + 1;
        while (j < n && (keys[j].hi >> 32) == (keys[i].hi >> 32)) ++j;
        if (j - i > 1) std::sort(keys.begin() + (long)i, keys.begin() + (long)j, greater);
        i = j;
    }
}

// pafPtrIntoVector + pafVectorIntoPeopleVector (GPU path): every connection of every pair sorted
// once by paf + 0.1 (score A + score B), then people are created, extended or merged
void people_global_sort(People& people, AssemblyScratch& sc, const PoseModelInfo& m,
                        const float* peaks, int max_peaks, const PairScores& scores)
{
    const int P = m.parts;
    const int stride = 3 * (max_peaks + 1);
    // std::greater on the reference's (total, paf, pair, i, j) tuple == descending packed keys
    std::vector<AssemblyScratch::Key>& conn = sc.keys;
    conn.clear();
    // s > 1e-6 (a double compare in the reference) == s >= thr for every float s (NaN fails both)
    const float thr = kPafMinFloat;
#if defined(__SSE__)
    const __m128 vthr = _mm_set1_ps(thr);
#endif
    for (int q = 0; q < m.npairs(); ++q) {
        const int pa = m.pairs[2 * q], pb = m.pairs[2 * q + 1];
        const int na = round_pos(peaks[pa * stride]);
        const int nb = round_pos(peaks[pb * stride]);
        for (int i = 1; i <= na; ++i) {
            const float* r = scores.row(q, i, nb);
            const float sa = 0.1f * peaks[pa * stride + i * 3 + 2];
            auto take = [&](int j0) {   // 0-based column
                const float s = r[j0];
                const float total = s + sa + 0.1f * peaks[pb * stride + (j0 + 1) * 3 + 2];
                conn.push_back({(uint64_t)ordered_bits(total) << 32 | ordered_bits(s),
                                (uint64_t)q << 32 | (uint64_t)i << 16 | (uint64_t)(j0 + 1)});
            };
            int j = 0;
#if defined(__SSE__)
            for (; j + 4 <= nb; j += 4) {   // 4 scores per compare; most fail
                unsigned mk = (unsigned)_mm_movemask_ps(_mm_cmpge_ps(_mm_loadu_ps(r + j), vthr));
                while (mk) {
                    take(j + __builtin_ctz(mk));
                    mk &= mk - 1;
                }
            }
#endif
            for (; j < nb; ++j)
                if (r[j] >= thr) take(j);
        }
    }
    sort_descending(conn, sc.keys_tmp);

    std::vector<int>& owner = sc.owner;   // person holding (part, peak)
    owner.assign((size_t)P * max_peaks, -1);
    std::vector<int>& dead = sc.dead;
    dead.clear();
    // the filled parts of each person as an intrusive list (node = a part, in a shared pool), so
    // a merge costs the merged-away person's parts instead of three sweeps over all P parts (a
    // BODY_135 frame of 20 people builds ~750 fragments and merges ~600 of them)
    std::vector<int>&node_part = sc.node_part, &node_next = sc.node_next, &head = sc.head,
    &tail = sc.tail;
    node_part.clear();
    node_next.clear();
    head.clear();
    tail.clear();
    auto link = [&](int p, int part) {
        const int nd = (int)node_part.size();
        node_part.push_back(part);
        node_next.push_back(-1);
        if (tail[p] < 0) head[p] = nd;
        else node_next[tail[p]] = nd;
        tail[p] = nd;
    };
    for (const AssemblyScratch::Key& c : conn) {
        const int q = (int)(c.lo >> 32), ci = (int)(c.lo >> 16 & 0xffff), cj = (int)(c.lo & 0xffff);
        const float paf = from_ordered_bits((uint32_t)c.hi);
        const int pa = m.pairs[2 * q], pb = m.pairs[2 * q + 1];
        const int sa = pa * stride + ci * 3 + 2, sb = pb * stride + cj * 3 + 2;
        int& oa = owner[(size_t)pa * max_peaks + ci - 1];
        int& ob = owner[(size_t)pb * max_peaks + cj - 1];
        if (oa < 0 && ob < 0) {            // 1. new person
            const int p = people.add();
            head.push_back(-1);
            tail.push_back(-1);
            people.row(p)[pa] = sa;
            people.row(p)[pb] = sb;
            link(p, pa);
            link(p, pb);
            people.found[p] = 2;
            people.score[p] = peaks[sa] + peaks[sb] + paf;
            oa = ob = p;
        } else if ((oa < 0) != (ob < 0)) {   // 2./3. extend the person holding one end
            const int p = oa >= 0 ? oa : ob;
            const int part2 = oa >= 0 ? pb : pa, s2 = oa >= 0 ? sb : sa;
            if (people.row(p)[part2] == 0) {
                people.row(p)[part2] = s2;
                link(p, part2);
                people.found[p]++;
                people.score[p] += peaks[s2] + paf;
                (oa >= 0 ? ob : oa) = p;
            }
        } else if (oa == ob) {               // 4. redundant connection inside one person
            people.score[oa] += paf;
        } else {                             // 5. merge two people with disjoint parts
            const int p1 = std::min(oa, ob), p2 = std::max(oa, ob);
            int* r1 = people.row(p1);
            const int* r2 = people.row(p2);
            // the parts of p2 are exactly the non-zero entries of its row: disjoint iff p1 holds
            // none of them, and then filling p1's empty entries from p2 copies exactly those
            bool disjoint = true;
            for (int nd = head[p2]; nd >= 0 && disjoint; nd = node_next[nd])
                disjoint = r1[node_part[nd]] == 0;
            if (!disjoint) continue;
            for (int nd = head[p2]; nd >= 0; nd = node_next[nd]) {
                const int k = node_part[nd];
                r1[k] = r2[k];
                // a (part, peak) slot's owner is set when, and only when, the slot enters a
                // row: re-point p2's slots to p1
                owner[(size_t)k * max_peaks + (r2[k] - k * stride - 2) / 3 - 1] = p1;
            }
            node_next[tail[p1]] = head[p2];
            tail[p1] = tail[p2];
            head[p2] = tail[p2] = -1;
            people.found[p1] += people.found[p2];
            people.score[p1] += people.score[p2] + paf;
            dead.push_back(p2);
        }
    }
    if (!dead.empty()) {   // erase merged-away people in place, keeping the order of the others
        std::sort(dead.begin(), dead.end());
        dead.erase(std::unique(dead.begin(), dead.end()), dead.end());
        size_t d = 0;
        int k = 0;
        for (int p = 0; p < people.size(); ++p) {
            if (d < dead.size() && dead[d] == p) { ++d; continue; }
            if (k != p) {
                std::copy(people.row(p), people.row(p) + P, people.row(k));
                people.found[k] = people.found[p];
                people.score[k] = people.score[p];
            }
            ++k;
        }
        people.slot.resize((size_t)k * P);
        people.found.resize(k);
        people.score.resize(k);
    }
}

// getRoiDiameterAndBounds (bodyPartConnectorBase.cpp:98-154): x, y, width, height
struct Roi {
    float x, y, w, h;
};
void roi_and_bounds(Roi& r, int& first, int& last, const int* row, const float* peaks, int from,
                    int to, float margin)
{
    r = {std::numeric_limits<float>::max(), std::numeric_limits<float>::max(), 0.f, 0.f};
    first = last = -1;
    for (int k = from; k < to; ++k) {
        const int s = row[k];
        if (s <= 0 || !(peaks[s] > 0)) continue;
        const float x = peaks[s - 2], y = peaks[s - 1];
        if (r.x > x) r.x = x;
        if (r.y > y) r.y = y;
        if (r.w < x) r.w = x;
        if (r.h < y) r.h = y;
        if (first < 0) first = k;
        last = k;
    }
    if (last > -1) {
        const float mx = r.w * margin, my = r.h * margin;
        r.x -= mx;
        r.y -= my;
        r.w += 2 * mx;
        r.h += 2 * my;
        ++last;
        r.w += 1 - r.x;
        r.h += 1 - r.y;
    }
}

// getKeypointsRoi (utilities/keypoint.cpp:586-632): intersection over union of two boxes after
// shifting both so that neither has a negative corner
float roi_overlap(Roi a, Roi b)
{
    const float bx = std::min(std::min(0.f, a.x), b.x);
    if (bx != 0) { a.x -= bx; b.x -= bx; }
    const float by = std::min(std::min(0.f, a.y), b.y);
    if (by != 0) { a.y -= by; b.y -= by; }
    const float x0 = std::max(a.x, b.x), y0 = std::max(a.y, b.y);
    const float x1 = std::min(a.x + a.w, b.x + b.w), y1 = std::min(a.y + a.h, b.y + b.h);
    if (!(x0 < x1 && y0 < y1)) return 0.f;
    const float inter = (x1 - x0) * (y1 - y0);
    return inter / (a.w * a.h + b.w * b.h - inter);
}

// getKeypointCounter (bodyPartConnectorBase.cpp:77-96)
void discount(int& counter, const int* row, int from, int to, int minimum)
{
    int k = 0;
    for (int i = from; i < to; ++i) k += row[i] > 0;
    if (k > minimum) counter += minimum - k;
}

// removePeopleBelowThresholdsAndFillFaces (bodyPartConnectorBase.cpp:720-884)
void select_people(std::vector<int>& keep, People& people, const float* peaks,
                   const ConnectParams& prm, bool maxpos)
{
    const int P = people.parts;
    keep.clear();
    std::vector<int> face_valid, face_invalid;
    for (int p = 0; p < people.size(); ++p) {
        const int* r = people.row(p);
        int counter = people.found[p];
        if (P >= 135) {   // hands and face count once each
            const int before = counter;
            discount(counter, r, 65, 135, 1);
            if (counter == 1) {
                face_invalid.push_back(p);
                continue;
            }
            if (counter != before) face_valid.push_back(p);
            discount(counter, r, 45, 65, 1);
            discount(counter, r, 25, 45, 1);
        }
        if (!maxpos && (P == 25 || P > 70)) {   // feet do not count
            const int before = counter;
            discount(counter, r, 19, 25, 0);
            if (counter != before && counter <= 4) continue;
        }
        if (counter >= prm.min_subset_cnt && (people.score[p] / counter) >= prm.min_subset_score)
            keep.push_back(p);
        else if ((counter < 1 && P != 25 && P < 70) || counter < 0)
            throw Error(1, "Bad personCounter (" + std::to_string(counter) +
                               "). Bug in this function if this happens.");
    }
    if (!keep.empty()) {   // face-only fragments join the best-overlapping valid face
        // each valid face's box, recomputed only after a fragment merged into it (the reference
        // recomputes it for every comparison; between merges it cannot change)
        std::vector<Roi> vroi(face_valid.size());
        std::vector<char> vstale(face_valid.size(), 1);
        for (int bad : face_invalid) {
            Roi rb;
            int fb, lb;
            roi_and_bounds(rb, fb, lb, people.row(bad), peaks, 65, 135, 0.2f);
            float best = 0.f;
            int besti = -1;
            for (int v = 0; v < (int)face_valid.size(); ++v) {
                if (vstale[v]) {
                    int fv, lv;
                    roi_and_bounds(vroi[v], fv, lv, people.row(face_valid[v]), peaks, 65, 135, 0.1f);
                    vstale[v] = 0;
                }
                const float o = roi_overlap(vroi[v], rb);
                if (best < o) {
                    best = o;
                    besti = v;
                }
            }
            if (!(best > 0.3f || (best > 0.01f && face_valid.size() < 3))) continue;
            const int good = face_valid[besti];
            vstale[besti] = 1;
            int* g = people.row(good);
            const int* src = people.row(bad);
            for (int k = fb; k < lb; ++k) {
                if (src[k] == 0) continue;
                const float si = peaks[src[k]];
                if (g[k] == 0) {
                    g[k] = src[k];
                    people.score[good] += si;
                } else if (peaks[g[k]] < si) {
                    people.score[good] += si - peaks[g[k]];
                    g[k] = src[k];
                }
            }
        }
    }
    if (keep.empty() && !maxpos) select_people(keep, people, peaks, prm, true);
}

}  // namespace

int assemble_people(const PoseModelInfo& m, const float* peaks, int max_peaks,
                    const PairScores& scores, const ConnectParams& prm, std::vector<float>& kp,
                    std::vector<float>& ks, AssemblyScratch* scratch)
{
    const int P = m.parts;
    AssemblyScratch local;
    AssemblyScratch& sc = scratch ? *scratch : local;
    People people(P, sc);
    if (prm.semantics == kConnectGpu) {
        people_global_sort(people, sc, m, peaks, max_peaks, scores);
    } else {
        if (!m.cpu_connector())   // bodyPartConnectorBase.cpp:165-167
            throw Error(4, std::string("connectBodyPartsCpu: only BODY_25, COCO_18 and MPI_15 are "
                                       "supported (") + m.name + "); use the GPU-path semantics");
        people_per_pair(people, m, peaks, max_peaks, scores);
    }
    std::vector<int>& keep = sc.keep;
    select_people(keep, people, peaks, prm, prm.maximize_positives);
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
