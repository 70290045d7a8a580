# Round-5 GPU study (profiles/r5k, part 2): kernel traces of 2 and 4 LSTM tenants placed one
# per socket / two per socket - where does the 4-tenant aggregate go?
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r5k
mkdir -p $O
for n in 2 4; do
  timeout -k 10 300 python3 -u tools/probe/cotenancy.py --case lstm-inf --procs $n --seconds 4 --placement split \
    --trace /tmp/r5k_tr$n > $O/traced_split$n.json 2> $O/traced_split$n.err || exit $?
  python3 tools/probe/cotenancy.py --analyze /tmp/r5k_tr$n > $O/overlap_split$n.json || exit $?
  tail -1 $O/traced_split$n.json | cut -c1-300
  cat $O/overlap_split$n.json
done
