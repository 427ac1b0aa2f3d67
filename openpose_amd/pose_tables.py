"""BODY_25 pose tables and default thresholds (host-side mirror of op::poseParameters).

/root/reference/src/openpose/pose/poseParameters.cpp:
  POSE_MAP_INDEX (BODY_25)          :253-256
  POSE_BODY_PART_PAIRS (BODY_25)    :417-419
  POSE_NUMBER_BODY_PARTS            :413-415
  default thresholds                :677-756
/root/reference/include/openpose/pose/poseParameters.hpp:14  POSE_MAX_PEOPLE = 127
"""
BODY25_PARTS = 25
BODY25_PAIRS = (1, 8, 1, 2, 1, 5, 2, 3, 3, 4, 5, 6, 6, 7, 8, 9, 9, 10, 10, 11, 8, 12, 12, 13, 13, 14,
                1, 0, 0, 15, 15, 17, 0, 16, 16, 18, 2, 17, 5, 18, 14, 19, 19, 20, 14, 21, 11, 22,
                22, 23, 11, 24)
BODY25_MAP_IDX = (0, 1, 14, 15, 22, 23, 16, 17, 18, 19, 24, 25, 26, 27, 6, 7, 2, 3, 4, 5, 8, 9, 10,
                  11, 12, 13, 30, 31, 32, 33, 36, 37, 34, 35, 38, 39, 20, 21, 28, 29, 40, 41, 42, 43,
                  44, 45, 46, 47, 48, 49, 50, 51)
BODY25_NUM_PAIRS = len(BODY25_PAIRS) // 2
POSE_MAX_PEOPLE = 127
NET_DECREASE_FACTOR = 8

# PoseModel enum values (include/openpose/pose/enumClasses.hpp:9-30); the tables of every model
# are in libopk_hip (api.pose_model_info)
BODY_25, COCO_18, MPI_15, MPI_15_4 = 0, 1, 2, 3
BODY_25B, BODY_135 = 13, 14

# connector semantics (include/opk.h): connectBodyPartsCpu / connectBodyPartsGpu assembly
CONNECT_CPU, CONNECT_GPU = 0, 1

# defaults (maximizePositives = false)
NMS_THRESHOLD = 0.05
CONNECT_INTER_MIN_ABOVE_THRESHOLD = 0.95
CONNECT_INTER_THRESHOLD = 0.05
CONNECT_MIN_SUBSET_CNT = 3
CONNECT_MIN_SUBSET_SCORE = 0.4
