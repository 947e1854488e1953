#!/bin/bash
# Load balance of the round-robin block shards (one gpurun call): every shard of N = 8 timed on one
# MI355X (tools/shard_sim.py --all), for the 8-GPU config C5 (david 1920x1080) and the headline C2
# (cornell 800x800x256), plus the N = 1 frame each is compared with. Outputs under gpurun_out/.
#   SPP_C5 (default 64): samples per pixel of the C5 frames (BASELINE C5 is 1024; Msamples/s is
#   ~spp-invariant at >= 64 spp, and the shard-to-shard spread is what this measures)
set -u
REPO=${GRAFT_REPO_ROOT:-$(pwd)}; OUT=$REPO/gpurun_out; mkdir -p "$OUT"; cd "$REPO"
TAG=${TAG:-r04}
SPP_C5=${SPP_C5:-64}
run() {
  local name=$1 limit=$2; shift 2
  timeout -k 10 "$limit" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"; tail -n ${TAILN:-12} "$OUT/$name.log"
  [ $rc -eq 0 ] || { echo "stopping after rc=$rc"; exit $rc; }
}
run ${TAG}_c5_shard_all_n8 600 python3 -u tools/shard_sim.py --scene david --w 1920 --h 1080 --spp $SPP_C5 --n 1,8 --all
run ${TAG}_c2_shard_all_n8 600 python3 -u tools/shard_sim.py --scene cornell-box --w 800 --h 800 --spp 256 --n 1,8 --all
echo ALL_OK
