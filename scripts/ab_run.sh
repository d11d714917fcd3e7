# A/B timing of library variants nusiprop_amd/libnusi_<v>.so: bash scripts/ab_run.sh <tag> <variant>...
# (C4 scan stage times + flux sha1, scripts/dev_scan_timing.py)
OUT=gpurun_out/$1; shift
mkdir -p $OUT
for v in "$@"; do
  NUSIPROP_LIB=$PWD/nusiprop_amd/libnusi_$v.so REPS=5 timeout -k 10 120 python scripts/dev_scan_timing.py 1024 300 > $OUT/c4_$v.log 2>&1 || exit 1
done
