#!/bin/bash
# scripts/r04_route_sweep.sh -- round 4: what each backend costs per wave size,
# in wall time and in host CPU time (VERDICT r03 "weak" item 8: where -n makes
# the GPU pay).  multipart_harness uploads a 256 x 10 MiB file (every part
# golden) through a pinned pool of -n buffers, no pipeline (one wave = -n parts),
# uploads that return at once, second pass reported; the backend forced to the
# gfx950 kernels (gpu), to the library's CPU MD5 (cpu: AVX-512 lanes from 8
# parts), or routed (auto, and auto with QSMD5_ROUTE_LANES=1).  cpu_s is the
# process's user + system time for the pass (getrusage), gather included.
# One JSON line per run in gpurun_out/r04_route_sweep.jsonl.
set -euo pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out
mkdir -p "$O"
cd "$R"
H=tests/cpp/multipart_harness
OUT=$O/r04_route_sweep.jsonl
: > "$OUT"
MiB=$((1 << 20))
run() {  # label, env assignment, args...
  local label=$1 envs=$2
  shift 2
  echo "== $label $envs $*" >&2
  timeout -k 10 180 env $envs "$H" "$@" > "$O/r04_one.json"
  python3 - "$label" "$O/r04_one.json" "$OUT" <<'EOF'
import json, sys
label, src, dst = sys.argv[1:4]
r = json.load(open(src))
gold = json.load(open("tests/golden/batch_10MiB.json"))["md5"]
r["golden_ok"] = all(m == gold[:r["parts"]] for m in r["md5_files"])
r["label"] = label
for k in ("md5", "md5_files", "part_sizes"):
    r.pop(k, None)
open(dst, "a").write(json.dumps(r) + "\n")
gib = r["size"] * r["files"] / 2.0 ** 30
print("%-28s waves %3d gpu %3d cpu %3d  %.2f GiB/s  cpu_s %.3f  golden %s" % (
    label, r["waves"], r["gpu_waves"], r["cpu_waves"], gib / r["wall_s_runs"][-1], r["cpu_s_runs"][-1],
    r["golden_ok"]), flush=True)
EOF
}
for n in 8 16 32 64 128 256; do
  for mode in gpu cpu auto lanes; do
    case $mode in
      gpu) envs="QSMD5_BACKEND=gpu" ;;
      cpu) envs="QSMD5_BACKEND=cpu" ;;
      auto) envs="QSMD5_BACKEND=auto" ;;
      lanes) envs="QSMD5_BACKEND=auto QSMD5_ROUTE_LANES=1" ;;
    esac
    run "n${n}_${mode}" "$envs" --aligned --size=$((256 * 10 * MiB)) --pool=$n --pinned --slab \
      --repeat=2 --no-pipeline
  done
done
echo "route sweep done: $OUT" >&2
