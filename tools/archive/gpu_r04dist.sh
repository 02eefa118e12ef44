#!/bin/bash
# r04: the process-group path on one GPU (RCCL world of 1 through torch.distributed.run, --dist), and the
# launcher's refusal of --gpus 2 on a one-GPU box
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
O=gpurun_out/${TAG:-r04dist}
mkdir -p $O
timeout -k 10 400 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29533 \
  bench.py --gpus 1 --dist --no-cpu --no-e2e > $O/dist_rehearsal_c2.json 2> $O/dist_rehearsal_c2.err || { echo "dist rehearsal failed"; tail -5 $O/dist_rehearsal_c2.err; exit 1; }
tail -1 $O/dist_rehearsal_c2.json | cut -c1-400
timeout -k 10 120 python3 bench.py --gpus 2 --no-cpu --no-e2e > $O/gpus2.out 2> $O/gpus2.err; rc=$?
echo "--gpus 2 on a one-GPU box: exit $rc"; tail -2 $O/gpus2.err
[ $rc -eq 2 ] || exit 1
