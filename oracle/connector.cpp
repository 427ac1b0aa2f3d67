// connector.cpp -- CPU oracle: PAF scoring + people assembly (TEST INFRASTRUCTURE, see oracle.h).
//
// Restates, from /root/reference/src/openpose/net/bodyPartConnectorBase.cpp:
//   getScoreAB                                :12-75    (PAF line integral, CPU clamp rules)
//   createPeopleVector                        :156-472  (per-pair greedy matching, CPU path)
//   pafPtrIntoVector / pafVectorIntoPeopleVector :474-718 (global-sort assembly, CUDA path)
//   removePeopleBelowThresholdsAndFillFaces   :720-884
//   peopleVectorToPeopleArray                 :886-934
//   connectBodyPartsCpu                       :1327-1377
// and the pose tables of /root/reference/src/openpose/pose/poseParameters.cpp:253-256,413-419.
// Pinned against the reference's own compiled code: tests/test_oracle_ref.py (oracle/_ref).
// Compiled with -ffp-contract=off (the reference CPU build has no FMA contraction).
#include <algorithm>
#include <cmath>
#include <functional>
#include <limits>
#include <set>
#include <tuple>
#include <vector>
#include "oracle.h"

namespace {

// ---- pose tables -------------------------------------------------------------------------
const unsigned kBody25Pairs[] = {1,8, 1,2, 1,5, 2,3, 3,4, 5,6, 6,7, 8,9, 9,10, 10,11, 8,12, 12,13,
    13,14, 1,0, 0,15, 15,17, 0,16, 16,18, 2,17, 5,18, 14,19, 19,20, 14,21, 11,22, 22,23, 11,24};
const unsigned kBody25Map[] = {0,1, 14,15, 22,23, 16,17, 18,19, 24,25, 26,27, 6,7, 2,3, 4,5, 8,9,
    10,11, 12,13, 30,31, 32,33, 36,37, 34,35, 38,39, 20,21, 28,29, 40,41, 42,43, 44,45, 46,47,
    48,49, 50,51};
const unsigned kCocoPairs[] = {1,2, 1,5, 2,3, 3,4, 5,6, 6,7, 1,8, 8,9, 9,10, 1,11, 11,12, 12,13,
    1,0, 0,14, 14,16, 0,15, 15,17, 2,16, 5,17};
const unsigned kCocoMap[] = {12,13, 20,21, 14,15, 16,17, 22,23, 24,25, 0,1, 2,3, 4,5, 6,7, 8,9,
    10,11, 28,29, 30,31, 34,35, 32,33, 36,37, 18,19, 26,27};
const unsigned kMpiPairs[] = {0,1, 1,2, 2,3, 3,4, 1,5, 5,6, 6,7, 1,14, 14,8, 8,9, 9,10, 14,11,
    11,12, 12,13};
const unsigned kMpiMap[] = {0,1, 2,3, 4,5, 6,7, 8,9, 10,11, 12,13, 14,15, 16,17, 18,19, 20,21,
    22,23, 24,25, 26,27};

struct Model { int parts; int pairs; const unsigned* pair; const unsigned* map; };
bool get_model(int m, Model& out)
{
    switch (m) {
        case 0: out = {25, 26, kBody25Pairs, kBody25Map}; return true;
        case 1: out = {18, 19, kCocoPairs, kCocoMap}; return true;
        case 2: case 3: out = {15, 14, kMpiPairs, kMpiMap}; return true;
        default: return false;
    }
}

inline int round_pos(float a) { return int(a + 0.5f); }   // fastMath.hpp:29-32

// One person candidate: for every part the index of its score inside `peaks` (0 = absent),
// the number of parts found and the running score.
struct Person {
    std::vector<int> part;
    int found = 0;
    float score = 0.f;
};

// ---- getScoreAB ----------------------------------------------------------------------------
float score_ab(const float* a, const float* b, const float* mx, const float* my, int W, int H,
               float inter_th, float inter_min_above, float nms_th)
{
    const float vx = b[0] - a[0];
    const float vy = b[1] - a[1];
    const float vmax = std::max(std::abs(vx), std::abs(vy));
    const int n = std::max(5, std::min(25, round_pos(std::sqrt(5 * vmax))));
    const float norm = float(std::sqrt(vx * vx + vy * vy));
    if (!(norm > 1e-6)) return 0.f;
    const float ux = vx / norm, uy = vy / norm;
    const float stepx = vx / n, stepy = vy / n;
    float sum = 0.f;
    unsigned count = 0;
    for (int s = 0; s < n; ++s) {
        const int px = std::max(0, std::min(W - 1, round_pos(a[0] + s * stepx)));
        const int py = std::max(0, std::min(H - 1, round_pos(a[1] + s * stepy)));
        const long idx = (long)py * W + px;
        const float v = ux * mx[idx] + uy * my[idx];
        if (v > inter_th) { sum += v; ++count; }
    }
    if (count / float(n) > inter_min_above) return sum / count;
    const float dist = std::sqrt(vx * vx + vy * vy);
    const double near = std::sqrt((double)(W * H)) / 150;   // std::sqrt(int) -> double
    if (dist < near) return float(nms_th + 1e-6);
    return 0.f;
}

// ---- createPeopleVector ----------------------------------------------------------------------
// `score_of(q, i, j)` returns the PAF score of pair q between 1-based peaks i of A and j of B.
template <class ScoreFn>
std::vector<Person> people_per_pair_greedy(const float* peaks, const Model& md, int max_peaks,
                                           ScoreFn score_of)
{
    std::vector<Person> people;
    const int stride = 3 * (max_peaks + 1);
    auto slot = [&](int part, int i) { return part * stride + i * 3 + 2; };
    auto new_person = [&](void) { Person p; p.part.assign(md.parts, 0); return p; };
    for (int q = 0; q < md.pairs; ++q) {
        const int pa = (int)md.pair[2 * q], pb = (int)md.pair[2 * q + 1];
        const int na = round_pos(peaks[pa * stride]);
        const int nb = round_pos(peaks[pb * stride]);
        if (na == 0 || nb == 0) {
            // one side empty: every candidate of the other side becomes a 1-part person
            const int part = (na == 0) ? pb : pa;
            const int cnt = (na == 0) ? nb : na;
            for (int i = 1; i <= cnt; ++i) {
                const int s = slot(part, i);
                bool dup = false;
                if (md.parts != 15)
                    for (const auto& p : people)
                        if (p.part[part] == s) { dup = true; break; }
                if (dup) continue;
                Person p = new_person();
                p.part[part] = s;
                p.found = 1;
                p.score = peaks[s];
                people.push_back(std::move(p));
            }
            continue;
        }
        // all candidate connections, best first: std::greater on (score, i, j)
        std::vector<std::tuple<double, int, int>> cand;
        for (int i = 1; i <= na; ++i)
            for (int j = 1; j <= nb; ++j) {
                const float s = score_of(q, i, j);
                if (s > 1e-6) cand.emplace_back(s, i, j);
            }
        std::sort(cand.begin(), cand.end(), std::greater<std::tuple<double, int, int>>());
        // greedy one-to-one selection, at most min(na, nb) connections
        std::vector<std::tuple<int, int, double>> chosen;
        {
            std::vector<char> usedA(na, 0), usedB(nb, 0);
            const int limit = std::min(na, nb);
            for (const auto& c : cand) {
                const int i = std::get<1>(c), j = std::get<2>(c);
                if (usedA[i - 1] || usedB[j - 1]) continue;
                chosen.emplace_back(slot(pa, i), slot(pb, j), std::get<0>(c));
                if ((int)chosen.size() == limit) break;
                usedA[i - 1] = 1;
                usedB[j - 1] = 1;
            }
        }
        if (chosen.empty()) continue;
        const bool ear_pair = (md.parts == 18 && (q == 17 || q == 18))
            || ((md.parts == 19 || md.parts == 25 || md.parts == 59 || md.parts == 65)
                && (q == 18 || q == 19));
        if (q == 0) {
            // the first pair seeds the people list
            for (const auto& c : chosen) {
                Person p = new_person();
                p.part[md.pair[0]] = std::get<0>(c);
                p.part[md.pair[1]] = std::get<1>(c);
                p.found = 2;
                p.score = float(peaks[std::get<0>(c)] + peaks[std::get<1>(c)] + std::get<2>(c));
                people.push_back(std::move(p));
            }
        } else if (ear_pair) {
            // ear pairs only fill a missing end of an existing person; counts/scores untouched
            for (const auto& c : chosen)
                for (auto& p : people) {
                    if (p.part[pa] == std::get<0>(c) && p.part[pb] == 0) p.part[pb] = std::get<1>(c);
                    else if (p.part[pb] == std::get<1>(c) && p.part[pa] == 0) p.part[pa] = std::get<0>(c);
                }
        } else {
            for (const auto& c : chosen) {
                const int ia = std::get<0>(c), ib = std::get<1>(c);
                const float sc = float(std::get<2>(c));
                bool attached = false;
                for (auto& p : people)
                    if (p.part[pa] == ia) {
                        p.part[pb] = ib;
                        p.found++;
                        p.score += peaks[ib] + sc;
                        attached = true;
                        break;
                    }
                if (attached) continue;
                Person p = new_person();
                p.part[pa] = ia;
                p.part[pb] = ib;
                p.found = 2;
                p.score = float(peaks[ia] + peaks[ib] + std::get<2>(c));
                people.push_back(std::move(p));
            }
        }
    }
    return people;
}

// ---- pafPtrIntoVector + pafVectorIntoPeopleVector (CUDA-path assembly) ----------------------
std::vector<Person> people_global_sort(const float* peaks, const Model& md, int max_peaks,
                                       const float* pair_scores)
{
    const int stride = 3 * (max_peaks + 1);
    std::vector<std::tuple<float, float, int, int, int>> conn;
    for (int q = 0; q < md.pairs; ++q) {
        const int pa = (int)md.pair[2 * q], pb = (int)md.pair[2 * q + 1];
        const int na = round_pos(peaks[pa * stride]);
        const int nb = round_pos(peaks[pb * stride]);
        const float* blk = pair_scores + (long)q * max_peaks * max_peaks;
        for (int i = 0; i < na; ++i)
            for (int j = 0; j < nb; ++j) {
                const float s = blk[i * max_peaks + j];
                if (!(s > 1e-6)) continue;
                const float total = s + 0.1f * peaks[pa * stride + (i + 1) * 3 + 2]
                                       + 0.1f * peaks[pb * stride + (j + 1) * 3 + 2];
                conn.emplace_back(total, s, q, i + 1, j + 1);
            }
    }
    std::sort(conn.begin(), conn.end(), std::greater<std::tuple<float, float, int, int, int>>());

    std::vector<Person> people;
    std::vector<int> owner((size_t)md.parts * max_peaks, -1);
    std::set<int, std::greater<int>> dead;
    for (const auto& c : conn) {
        const float paf = std::get<1>(c);
        const int q = std::get<2>(c), i = std::get<3>(c), j = std::get<4>(c);
        const int pa = (int)md.pair[2 * q], pb = (int)md.pair[2 * q + 1];
        const int sa = (pa * (max_peaks + 1) + i) * 3 + 2;
        const int sb = (pb * (max_peaks + 1) + j) * 3 + 2;
        int& oa = owner[(size_t)pa * max_peaks + i - 1];
        int& ob = owner[(size_t)pb * max_peaks + j - 1];
        if (oa < 0 && ob < 0) {
            Person p; p.part.assign(md.parts, 0);
            p.part[pa] = sa; p.part[pb] = sb; p.found = 2;
            p.score = float(peaks[sa] + peaks[sb] + paf);
            oa = ob = (int)people.size();
            people.push_back(std::move(p));
        } else if ((oa >= 0) != (ob >= 0)) {
            const int who = oa >= 0 ? oa : ob;
            int& other = oa >= 0 ? ob : oa;
            const int part2 = oa >= 0 ? pb : pa;
            const int s2 = oa >= 0 ? sb : sa;
            Person& p = people[who];
            if (p.part[part2] == 0) {
                p.part[part2] = s2;
                p.found++;
                p.score += peaks[s2] + paf;
                other = who;
            }
        } else if (oa == ob) {
            people[oa].score += paf;
        } else {
            const int keep = std::min(oa, ob), drop = std::max(oa, ob);
            Person& p1 = people[keep];
            const Person& p2 = people[drop];
            bool disjoint = true;
            for (int k = 0; k < md.parts; ++k)
                if (p1.part[k] > 0 && p2.part[k] > 0) { disjoint = false; break; }
            if (disjoint) {
                for (int k = 0; k < md.parts; ++k)
                    if (p1.part[k] == 0) p1.part[k] = p2.part[k];
                p1.found += p2.found;
                p1.score += p2.score + paf;
                dead.insert(drop);
                for (auto& o : owner) if (o == drop) o = keep;
            }
        }
    }
    for (int d : dead) people.erase(people.begin() + d);
    return people;
}

// ---- removePeopleBelowThresholdsAndFillFaces --------------------------------------------------
struct Roi { float x, y, w, h; };
void roi_and_bounds(Roi& r, int& first, int& last, const Person& p, const float* peaks,
                    int from, int to, float margin)
{
    r = {std::numeric_limits<float>::max(), std::numeric_limits<float>::max(), 0.f, 0.f};
    first = last = -1;
    for (int k = from; k < to; ++k) {
        const int s = p.part[k];
        if (s > 0 && peaks[s] > 0) {
            const float x = peaks[s - 2], y = peaks[s - 1];
            if (r.x > x) r.x = x;
            if (r.y > y) r.y = y;
            if (r.w < x) r.w = x;
            if (r.h < y) r.h = y;
            if (first < 0) first = k;
            last = k;
        }
    }
    if (last > -1) {
        const float mx = r.w * margin, my = r.h * margin;
        r.x -= mx; r.y -= my; r.w += 2 * mx; r.h += 2 * my;
        ++last;
        r.w += 1 - r.x;
        r.h += 1 - r.y;
    }
}

float roi_iou(const Roi& a0, const Roi& b0)   // keypoint.cpp:586-632 (getKeypointsRoi)
{
    Roi a = a0, b = b0;
    const float bx = std::min(std::min(0.f, a0.x), b0.x);
    if (bx != 0) { a.x -= bx; b.x -= bx; }
    const float by = std::min(std::min(0.f, a0.y), b0.y);
    if (by != 0) { a.y -= by; b.y -= by; }
    const float x0 = std::max(a.x, b.x), y0 = std::max(a.y, b.y);
    const float x1 = std::min(a.x + a.w, b.x + b.w), y1 = std::min(a.y + a.h, b.y + b.h);
    if (!(x0 < x1 && y0 < y1)) return 0.f;
    const float inter = (x1 - x0) * (y1 - y0);
    return float(inter) / float(a.w * a.h + b.w * b.h - inter);
}

int count_and_discount(int& counter, const Person& p, int from, int to, int minimum)
{
    int k = 0;
    for (int i = from; i < to; ++i) k += (p.part[i] > 0);
    if (k > minimum) counter += minimum - k;
    return counter;
}

void select_people(std::vector<int>& valid, int& npeople, std::vector<Person>& people, int parts,
                   int min_cnt, float min_score, bool maxpos, const float* peaks)
{
    npeople = 0;
    valid.clear();
    std::vector<int> face_valid, face_invalid;
    for (int i = 0; i < (int)people.size(); ++i) {
        int counter = people[i].found;
        if (parts >= 135) {
            const int before = counter;
            count_and_discount(counter, people[i], 65, 135, 1);
            if (counter == 1) { face_invalid.push_back(i); continue; }
            if (before != counter) face_valid.push_back(i);
            count_and_discount(counter, people[i], 45, 65, 1);
            count_and_discount(counter, people[i], 25, 45, 1);
        }
        if (!maxpos && (parts == 25 || parts > 70)) {
            const int before = counter;
            count_and_discount(counter, people[i], 19, 25, 0);
            if (counter != before && counter <= 4) continue;
        }
        const float sc = people[i].score;
        if (counter >= min_cnt && (sc / counter) >= min_score) {
            ++npeople;
            valid.push_back(i);
        }
    }
    if (npeople > 0) {
        for (int bad : face_invalid) {
            Roi rb; int fb, lb;
            roi_and_bounds(rb, fb, lb, people[bad], peaks, 65, 135, 0.2f);
            float best = 0.f; int besti = -1;
            for (int v = 0; v < (int)face_valid.size(); ++v) {
                Roi rv; int fv, lv;
                roi_and_bounds(rv, fv, lv, people[face_valid[v]], peaks, 65, 135, 0.1f);
                const float o = roi_iou(rv, rb);
                if (best < o) { best = o; besti = v; }
            }
            if (best > 0.3f || (best > 0.01f && face_valid.size() < 3)) {
                Person& good = people[face_valid[besti]];
                const Person& src = people[bad];
                for (int k = fb; k < lb; ++k) {
                    if (src.part[k] == 0) continue;
                    const float sv = good.part[k] ? peaks[good.part[k]] : 0.f;
                    const float si = peaks[src.part[k]];
                    if (good.part[k] == 0) { good.part[k] = src.part[k]; good.score += si; }
                    else if (sv < si) { good.part[k] = src.part[k]; good.score += si - sv; }
                }
            }
        }
    }
    if (npeople == 0 && !maxpos)
        select_people(valid, npeople, people, parts, min_cnt, min_score, true, peaks);
}

int write_people(float* kp, float* ks, int max_people, const std::vector<Person>& people,
                 const std::vector<int>& valid, const float* peaks, int parts, int pairs,
                 float scale)
{
    const float inv = 1 / float(parts + pairs);
    const int n = (int)valid.size();
    for (int o = 0; o < n && o < max_people; ++o) {
        const Person& p = people[valid[o]];
        for (int k = 0; k < parts; ++k) {
            float* d = kp + ((long)o * parts + k) * 3;
            const int s = p.part[k];
            if (s > 0) { d[0] = peaks[s - 2] * scale; d[1] = peaks[s - 1] * scale; d[2] = peaks[s]; }
            else { d[0] = d[1] = d[2] = 0.f; }
        }
        ks[o] = p.score * inv;
    }
    return n;
}

}  // namespace

extern "C" {

int orc_pose_num_parts(int m) { Model md; return get_model(m, md) ? md.parts : -1; }
int orc_pose_num_pairs(int m) { Model md; return get_model(m, md) ? md.pairs : -1; }
const unsigned* orc_pose_pairs(int m) { Model md; return get_model(m, md) ? md.pair : nullptr; }
const unsigned* orc_pose_map_idx(int m) { Model md; return get_model(m, md) ? md.map : nullptr; }

float orc_paf_score(const float* a, const float* b, const float* mx, const float* my, int W, int H,
                    float inter_th, float inter_min_above, float nms_th)
{
    return score_ab(a, b, mx, my, W, H, inter_th, inter_min_above, nms_th);
}

int orc_connect_body_parts(float* kp, float* ks, int max_people, const float* heat,
                           const float* peaks, int pose_model, int W, int H, int max_peaks,
                           float inter_min_above, float inter_th, int min_cnt, float min_score,
                           float nms_th, float scale, int maxpos)
{
    Model md;
    if (!get_model(pose_model, md)) return -1;
    const long area = (long)W * H;
    const int stride = 3 * (max_peaks + 1);
    const int base = md.parts + 1;   // + background channel
    auto fn = [&](int q, int i, int j) {
        const float* mx = heat + (base + md.map[2 * q]) * area;
        const float* my = heat + (base + md.map[2 * q + 1]) * area;
        const float* a = peaks + md.pair[2 * q] * stride + i * 3;
        const float* b = peaks + md.pair[2 * q + 1] * stride + j * 3;
        return score_ab(a, b, mx, my, W, H, inter_th, inter_min_above, nms_th);
    };
    auto people = people_per_pair_greedy(peaks, md, max_peaks, fn);
    std::vector<int> valid;
    int n = 0;
    select_people(valid, n, people, md.parts, min_cnt, min_score, maxpos != 0, peaks);
    return write_people(kp, ks, max_people, people, valid, peaks, md.parts, md.pairs, scale);
}

int orc_connect_from_scores(float* kp, float* ks, int max_people, const float* pair_scores,
                            const float* peaks, int pose_model, int max_peaks, int min_cnt,
                            float min_score, float scale, int maxpos)
{
    Model md;
    if (!get_model(pose_model, md)) return -1;
    auto fn = [&](int q, int i, int j) {
        return pair_scores[((long)q * max_peaks + (i - 1)) * max_peaks + (j - 1)];
    };
    auto people = people_per_pair_greedy(peaks, md, max_peaks, fn);
    std::vector<int> valid;
    int n = 0;
    select_people(valid, n, people, md.parts, min_cnt, min_score, maxpos != 0, peaks);
    return write_people(kp, ks, max_people, people, valid, peaks, md.parts, md.pairs, scale);
}

int orc_connect_gpu_semantics(float* kp, float* ks, int max_people, const float* pair_scores,
                              const float* peaks, int pose_model, int max_peaks, int min_cnt,
                              float min_score, float scale, int maxpos)
{
    Model md;
    if (!get_model(pose_model, md)) return -1;
    auto people = people_global_sort(peaks, md, max_peaks, pair_scores);
    std::vector<int> valid;
    int n = 0;
    select_people(valid, n, people, md.parts, min_cnt, min_score, maxpos != 0, peaks);
    return write_people(kp, ks, max_people, people, valid, peaks, md.parts, md.pairs, scale);
}

int orc_connect_gpu_tables(float* kp, float* ks, int max_people, const float* pair_scores,
                           const float* peaks, int parts, int npairs, const unsigned* pairs,
                           int max_peaks, int min_cnt, float min_score, float scale, int maxpos)
{
    const Model md{parts, npairs, pairs, nullptr};
    auto people = people_global_sort(peaks, md, max_peaks, pair_scores);
    std::vector<int> valid;
    int n = 0;
    select_people(valid, n, people, md.parts, min_cnt, min_score, maxpos != 0, peaks);
    return write_people(kp, ks, max_people, people, valid, peaks, md.parts, md.pairs, scale);
}

void orc_pair_scores(float* out, const float* heat, const float* peaks, int npairs,
                     const unsigned* pairs, const unsigned* mapx, const unsigned* mapy, int W,
                     int H, int max_peaks, float inter_th, float inter_min_above, float nms_th)
{
    const long area = (long)W * H;
    const int stride = 3 * (max_peaks + 1);
    for (int q = 0; q < npairs; ++q) {
        const float* a0 = peaks + pairs[2 * q] * stride;
        const float* b0 = peaks + pairs[2 * q + 1] * stride;
        const int na = round_pos(a0[0]), nb = round_pos(b0[0]);
        float* o = out + (long)q * max_peaks * max_peaks;
        for (int i = 0; i < max_peaks * max_peaks; ++i) o[i] = 0.f;
        for (int i = 0; i < na; ++i)
            for (int j = 0; j < nb; ++j)
                o[i * max_peaks + j] = score_ab(a0 + (i + 1) * 3, b0 + (j + 1) * 3,
                                                heat + mapx[q] * area, heat + mapy[q] * area, W, H,
                                                inter_th, inter_min_above, nms_th);
    }
}

}  // extern "C"
