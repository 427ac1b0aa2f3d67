// pose_model.cpp -- pose tables (/root/reference/src/openpose/pose/poseParameters.cpp:253-256,
// 413-419 for BODY_25; COCO_18 / MPI_15 / MPI_15_4 from the same arrays and
// include/openpose/pose/poseParametersRender.hpp:70-71).
#include "pose_model.h"

#include "../common.h"

namespace opk {

const PoseModelInfo& pose_model(int id)
{
    static const PoseModelInfo body25{0, 25, true,
        {1,8, 1,2, 1,5, 2,3, 3,4, 5,6, 6,7, 8,9, 9,10, 10,11, 8,12, 12,13, 13,14, 1,0, 0,15, 15,17,
         0,16, 16,18, 2,17, 5,18, 14,19, 19,20, 14,21, 11,22, 22,23, 11,24},
        {0,1, 14,15, 22,23, 16,17, 18,19, 24,25, 26,27, 6,7, 2,3, 4,5, 8,9, 10,11, 12,13, 30,31,
         32,33, 36,37, 34,35, 38,39, 20,21, 28,29, 40,41, 42,43, 44,45, 46,47, 48,49, 50,51}};
    static const PoseModelInfo coco18{1, 18, true,
        {1,2, 1,5, 2,3, 3,4, 5,6, 6,7, 1,8, 8,9, 9,10, 1,11, 11,12, 12,13, 1,0, 0,14, 14,16, 0,15,
         15,17, 2,16, 5,17},
        {12,13, 20,21, 14,15, 16,17, 22,23, 24,25, 0,1, 2,3, 4,5, 6,7, 8,9, 10,11, 28,29, 30,31,
         34,35, 32,33, 36,37, 18,19, 26,27}};
    static const std::vector<int> mpi_pairs{0,1, 1,2, 2,3, 3,4, 1,5, 5,6, 6,7, 1,14, 14,8, 8,9,
                                            9,10, 14,11, 11,12, 12,13};
    static const std::vector<int> mpi_map{0,1, 2,3, 4,5, 6,7, 8,9, 10,11, 12,13, 14,15, 16,17,
                                          18,19, 20,21, 22,23, 24,25, 26,27};
    static const PoseModelInfo mpi15{2, 15, true, mpi_pairs, mpi_map};
    static const PoseModelInfo mpi15_4{3, 15, true, mpi_pairs, mpi_map};
    switch (id) {
        case 0: return body25;
        case 1: return coco18;
        case 2: return mpi15;
        case 3: return mpi15_4;
        default: throw Error(4, "pose model " + std::to_string(id) + " has no tables in libopk_hip");
    }
}

}  // namespace opk
