# one line per bench log: ms_per_step, kernel_ms, value (scripts/summ.sh DIR)
for f in $1/*.log; do python3 - "$f" <<'PY'
import json, sys
f = sys.argv[1]
for l in open(f):
    if l.startswith('{'):
        d = json.loads(l)
        print(f.split('/')[-1], round(d['ms_per_step'], 3), round(d['roofline']['kernel_ms'], 3), '%.3g' % d['value'])
PY
done
