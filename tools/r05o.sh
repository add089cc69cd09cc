set -u
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out/r05o
timeout -k 10 400 python tools/api_leg.py > gpurun_out/r05o/api.json 2> gpurun_out/r05o/api.err || { tail -30 gpurun_out/r05o/api.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/r05o/api.json'));print(d['env_steps_per_s']);print(json.dumps(d['prompt_kernels'],indent=1))"
