# (round 6 experiment, with the CU-masked tree stream of gpu_r06_treecu.sh applied: removed, see profiles/r06/ab_tree_cumask/)
set -o pipefail
D="SM_LIB=stereomatch_amd/libstereomst_dev.so"
REPS=2 bash tools/gpu_ab.sh "q4base|$D|" "q8base|$D GPU_MAX_HW_QUEUES=8|" "q8cu64|$D GPU_MAX_HW_QUEUES=8 SM_TREE_CUS=64|" "q8cu128|$D GPU_MAX_HW_QUEUES=8 SM_TREE_CUS=128|" "q8cu256|$D GPU_MAX_HW_QUEUES=8 SM_TREE_CUS=256|"
