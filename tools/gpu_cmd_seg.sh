# accumulation-segment / reduction-segment sweep at 2^26
set -o pipefail
timeout -k 10 900 python3 tools/msm_ab.py 26 "" ECG_MSM_ACC_SEG=96 ECG_MSM_ACC_SEG=192 ECG_MSM_ACC_SEG=256 ECG_MSM_RED_SEG=32 ECG_MSM_RED_SEG=128
