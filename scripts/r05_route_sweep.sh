#!/bin/bash
# scripts/r05_route_sweep.sh -- round 5: does `auto` pick
# the faster backend, on an idle host and on a loaded one?  multipart_harness
# uploads a 256 x 10 MiB file (every part golden) through a pinned pool of -n
# buffers, no pipeline (one wave = -n parts), uploads that return at once; the
# process held to 4 cores (--cpus=4, the CPU backend's default 4 threads), with
# 0, 4 or 12 spinning threads of "qsfs work" on those cores (--load).  Backend
# forced to the gfx950 kernels (gpu), to the CPU (cpu: AVX-512 lanes from 8
# parts), or routed (auto, lanes priced and load feedback on: the round-5
# defaults).  Three passes; the third is reported (auto has seen the load by
# then).  One JSON line per run in gpurun_out/r05_route_sweep.jsonl.
set -euo pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out
mkdir -p "$O"
cd "$R"
H=tests/cpp/multipart_harness
OUT=$O/r05_route_sweep.jsonl
: > "$OUT"
MiB=$((1 << 20))
run() {  # label, env assignment, args...
  local label=$1 envs=$2
  shift 2
  timeout -k 10 180 env $envs "$H" "$@" > "$O/r05_one.json"
  python3 - "$label" "$O/r05_one.json" "$OUT" <<'EOF'
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
print("%-22s waves %3d gpu %3d cpu %3d  %6.2f GiB/s  eff %.2f  golden %s" % (
    label, r["waves"], r["gpu_waves"], r["cpu_waves"], gib / r["wall_s_runs"][-1], r["cpu_efficiency"],
    r["golden_ok"]), flush=True)
if not r["golden_ok"]:
    sys.exit(1)
EOF
}
for load in 0 4 12; do
  for n in 8 32 64 128 256; do
    for mode in gpu cpu auto; do
      run "load${load}_n${n}_${mode}" "QSMD5_BACKEND=$mode" --aligned --size=$((256 * 10 * MiB)) --pool=$n \
        --pinned --slab --repeat=3 --no-pipeline --cpus=4 --load=$load
    done
  done
done
echo "route sweep done: $OUT" >&2
