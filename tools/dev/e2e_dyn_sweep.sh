# end-to-end leg under tier-0 run settings and chunkings (bench.py --e2e-only); one line per setting
set -e
run() { echo "== $*"; env "$@" timeout -k 10 200 python -u bench.py --e2e-only --e2e-steps 8 2>/dev/null | grep "^{" | python -c "import json,sys; j=json.loads(sys.stdin.read())['end_to_end']; print(j['ms_per_batch'], j['tier0_ms_sum'], j['chunks'], j['rows_form']['ms_per_batch'])"; }
run KETO_X=0
run KETO_T0_DYN_FORCE=1
run KETO_T0_DYN_FORCE=1 KETO_CHUNK=8388608
run KETO_T0_DYN_FORCE=1 KETO_CHUNK=8388608 KETO_CHUNK_FIRST=2097152
run KETO_CHUNK=8388608 KETO_CHUNK_FIRST=2097152
run KETO_T0_DYN_FORCE=1 KETO_CHUNK=2097152
