set -u
cd "${GRAFT_REPO_ROOT}"
SKIP_API=1 bash tools/r05_check.sh r05ah "tests/test_gpu_token_turn.py" || exit $?
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > gpurun_out/r05ah/bench.json 2> gpurun_out/r05ah/bench.err
rc=$?; echo "[bench] rc=$rc"; [ $rc -ne 0 ] && { tail -20 gpurun_out/r05ah/bench.err; exit $rc; }
python - <<'PY'
import json
d = json.loads(open("gpurun_out/r05ah/bench.json").read().strip().splitlines()[-1])
print("value", d["value"], "ms_per_step", d["ms_per_step"])
t = d["text_api"]
print("token_rollout", {k: v for k, v in t["token_rollout"].items() if k.startswith("ms")})
print("detok_parse us", t["detok_parse"]["us"])
print("api", d.get("api_variant", {}).get("env_steps_per_s"))
PY
