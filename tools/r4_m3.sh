#!/bin/bash
# M3 (densifying, configs[2]): graph-replayed across the refine vs eager.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${1:-r4_m3}; mkdir -p $O
for r in 1 2; do
  timeout -k 10 400 python -u bench.py --config m3 --no-traffic --no-cpu-baseline > $O/graph.$r.json 2> $O/graph.$r.err || exit 1
  echo "graph $r $(python3 -c "import json;d=json.loads(open('$O/graph.$r.json').read().strip().splitlines()[-1]);print(round(d['value'],1), d['config']['step_issue'][:160], d['config']['densification'][-90:])")"
  timeout -k 10 400 python -u bench.py --config m3 --no-traffic --no-cpu-baseline --eager > $O/eager.$r.json 2> $O/eager.$r.err || exit 2
  echo "eager $r $(python3 -c "import json;d=json.loads(open('$O/eager.$r.json').read().strip().splitlines()[-1]);print(round(d['value'],1))")"
done
exit 0
