# NTT tile / threads-per-workgroup sweep (parity checked inside ntt_ab against parallel_fft)
set -o pipefail
timeout -k 10 900 python3 tools/ntt_ab.py "" ECG_NTT_EPT=8 ECG_NTT_TILE=11 ECG_NTT_TILE=11,ECG_NTT_EPT=8 ECG_NTT_TILE=9 ECG_NTT_TILE=9,ECG_NTT_EPT=8 ECG_NTT_MAXDEG=12 ECG_NTT_MAXDEG=12,ECG_NTT_EPT=8
