# Round 4 session 2: store-policy rows of launch_phases (fill / decode / copy), the
# TCP zip + sparse tests, the xGMI pool tests, the sparse parity tests + codec
# timing + kernel stats (tools/sp_gpu.sh), then the bench's local_reduce /
# copy_ceiling / sparse legs with the host-gap-free event windows.
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 240 ./tools/launch_phases 64,256 24 > gpurun_out/lp2.txt 2>&1 || { echo "launch_phases failed"; cat gpurun_out/lp2.txt; exit 1; }
cat gpurun_out/lp2.txt
timeout -k 10 300 python -u -m pytest tests/test_gpu_tcp.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread -k "zip or sparse" > gpurun_out/tcp_pytest.log 2>&1 || { tail -30 gpurun_out/tcp_pytest.log; exit 1; }
tail -2 gpurun_out/tcp_pytest.log
timeout -k 10 400 python -u -m pytest tests/test_gpu_xgmi.py -x -q -p no:cacheprovider --timeout 300 --timeout-method thread -k "recreate or release" > gpurun_out/xgmi_pytest.log 2>&1 || { tail -30 gpurun_out/xgmi_pytest.log; exit 1; }
tail -2 gpurun_out/xgmi_pytest.log
bash tools/sp_gpu.sh || exit 1
timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-host-fed --no-tcp-edge --xgmi-coresident 0 > gpurun_out/bench_s2.log 2>&1 || { tail -20 gpurun_out/bench_s2.log; exit 1; }
python3 - <<'PY'
import json
d = json.loads(open("gpurun_out/bench_s2.log").read().strip().splitlines()[-1])
print("value", d["value"], "roofline", {k: v for k, v in d["roofline"].items() if not isinstance(v, dict)})
for k in ("local_reduce", "copy_ceiling"):
    print(k, {a: (b.get("us_per_launch"), b.get("frac_of_hbm_peak")) if isinstance(b, dict) else b for a, b in d[k].items() if a not in ("workload", "timing", "hbm_peak_gbs")})
print("path_kernels", {a: b.get("frac_of_hbm_peak") for a, b in d["path_kernels"].items() if isinstance(b, dict)})
sc = d["sparse_codec"]
print("sparse drop", sc["drop"].get("stream_ms"), sc["drop"].get("stream_frac_of_hbm_peak"), "lift", sc["lift_dev"].get("stream_ms"), sc["lift_dev"].get("stream_frac_of_hbm_peak"))
PY
