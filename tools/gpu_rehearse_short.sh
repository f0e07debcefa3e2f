set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out/rehearse
GG_BENCH_DEVICE=0 timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 \
  bench.py --gpus 2 --steps 3 --warmup 1 --docs 100000 --dist-backend gloo --no-cpu-baseline > gpurun_out/rehearse/bench2.log 2>&1 || { tail -30 gpurun_out/rehearse/bench2.log; exit 1; }
grep '^{' gpurun_out/rehearse/bench2.log | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['detail']['rule_tallies_sum'], d['detail']['rule_tallies_fetched'])"
timeout -k 10 400 python bench.py --steps 3 --warmup 1 --docs 100000 --no-cpu-baseline > gpurun_out/rehearse/bench1.log 2>&1 || { tail -30 gpurun_out/rehearse/bench1.log; exit 1; }
tail -1 gpurun_out/rehearse/bench1.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['detail']['rule_tallies_sum'], d['detail']['rule_tallies_fetched'])"
