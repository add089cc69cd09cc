set -u
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out/r05ak
SKIP_API=1 bash tools/r05_check.sh r05ak "tests/test_gpu_token_turn.py" || exit $?
for v in "" variants/libragen_amd_tok_norender.so; do
  RAGEN_AMD_LIB=$v timeout -k 10 120 python -u tools/bench_token_turn.py >> gpurun_out/r05ak/ab.txt 2>> gpurun_out/r05ak/ab.err
  rc=$?; echo "[$v] rc=$rc"; [ $rc -ne 0 ] && { tail -5 gpurun_out/r05ak/ab.err; exit $rc; }
done
cat gpurun_out/r05ak/ab.txt
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > gpurun_out/r05ak/bench.json 2> gpurun_out/r05ak/bench.err
rc=$?; echo "[bench] rc=$rc"; [ $rc -ne 0 ] && { tail -20 gpurun_out/r05ak/bench.err; exit $rc; }
python - <<'PY'
import json
d = json.loads(open("gpurun_out/r05ak/bench.json").read().strip().splitlines()[-1])
print("value", d["value"], "ms_per_step", d["ms_per_step"])
t = d["text_api"]
print("token_rollout", {k: v for k, v in t["token_rollout"].items() if k.startswith("ms")})
print("api", d.get("api_variant", {}).get("env_steps_per_s"))
PY
