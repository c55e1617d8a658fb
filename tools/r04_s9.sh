# Round 4 session 9: the N > 1 bench flow rehearsed on one GPU (2 ranks, xGMI
# schedule on device 0, no RCCL): torchrun launch, gloo control plane, the line
# with nx_roofline's flat keys.
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 500 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 10 --warmup 3 --algo xgmi --same-device --alt-schedules "" --sweep-mib "1,64" > gpurun_out/rehearsal_n2.log 2>&1 || { tail -30 gpurun_out/rehearsal_n2.log; exit 1; }
grep '^{"metric"' gpurun_out/rehearsal_n2.log | tail -1 > gpurun_out/rehearsal_n2.json
python3 - <<'PY'
import json
d = json.load(open("gpurun_out/rehearsal_n2.json"))
print("value", d["value"], "n", d["n_gpus"], "check", d["check"])
print({k: v for k, v in d["roofline"].items() if not isinstance(v, dict)})
PY
