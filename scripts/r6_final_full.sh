# Round 6's whole-suite pass on the final library: smoke(), every GPU test, the bench at C1 / C2 /
# C5 / C4, the N > 1 launch paths over the gloo rehearsal transport (torchrun x2 and the
# self-launched x4 at C2, the self-launched x8 at C3 with its "link" record).
# usage: bash scripts/r6_final_full.sh TAG
set -u
TAG=${1:-r6full}
bash scripts/full_pass.sh $TAG || exit 1
cd "$GRAFT_REPO_ROOT" && O=gpurun_out/$TAG
timeout -k 10 500 python -u bench.py --gpus 8 --dist-backend gloo --config C3 --steps 2 --warmup 1 --timeout 420 \
  > $O/self8_C3.log 2>&1 || { echo "self8 C3 failed"; tail -5 $O/self8_C3.log; exit 1; }
python3 -c "
import json;l=[json.loads(x) for x in open('$O/self8_C3.log') if x.startswith('{')][-1]
print('self8 C3', l.get('verified'), json.dumps(l.get('link')))"
