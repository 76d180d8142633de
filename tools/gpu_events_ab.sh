set -o pipefail
cd "$GRAFT_REPO_ROOT"
for i in 1 2; do for e in 1 10; do
timeout -k 10 200 python3 bench.py --legs none --steps 4000 --warmup 20 --event-every $e > gpurun_out/ev.json 2>/dev/null || exit 1
python3 -c "
import json; d=json.loads(open('gpurun_out/ev.json').read().strip().splitlines()[-1])
print('every $e', d['ms_per_step'], d['roofline']['avg_kernel_ms'], d['value'], d['kernel_timing'])"
done; done
