set -u
mkdir -p gpurun_out/ab
for i in 1 2; do for w in 1 2 4; do
  RAGEN_AMD_LIB=$PWD/tools/_build/libragen_amd_wpb$w.so timeout -k 10 120 python bench.py --no-cpu-baseline --no-extras > gpurun_out/ab/wpb${w}_$i.log 2>&1 || { echo fail $w; tail -3 gpurun_out/ab/wpb${w}_$i.log; exit 1; }
  python3 -c "import json; l=[x for x in open('gpurun_out/ab/wpb${w}_$i.log') if x.startswith('{')][-1]; d=json.loads(l); print('wpb$w', round(d['ms_per_step']*1e3,2), 'us/step', round(d['roofline']['avg_launch_us'],2), 'us/launch')"
done; done
