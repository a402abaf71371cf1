for s in 1 2 3 4 5 6 7 8 9 10 11 12 13 14 15 16 17 18 19 20; do MIMIC=1 SEED=3 timeout -k 10 60 python bench/bncnn_first.py 2>&1 | grep '{' | python3 -c "
import sys,json
for l in sys.stdin:
    d=json.loads(l); bad={k:v for k,v in d.items() if k.startswith('diag')}; print(bad if bad else 'ok')" || exit 1; done
