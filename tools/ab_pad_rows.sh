mkdir -p gpurun_out/r04pad
for v in old pr1 pr1nt pr4c pr4nt old pr4c pr4nt; do
  RAGEN_AMD_LIB=$PWD/variants/libragen_amd_$v.so timeout -k 10 120 python tools/bench_pad_rows.py >> gpurun_out/r04pad/ab.txt 2>&1 || exit 1
done
