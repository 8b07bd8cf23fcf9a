cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/c3tl
for it in 1 2 4; do
  RP_MEMBERS_CK_ITEMS=$it timeout -s KILL 180 rocprofv3 --kernel-trace -d gpurun_out/c3tl/prof$it -o run -- python3 -u tools/c3_timeline.py run 128 > gpurun_out/c3tl/run$it.log 2>&1 || { echo prof failed; tail -20 gpurun_out/c3tl/run$it.log; exit 1; }
  db=$(find gpurun_out/c3tl/prof$it -name '*.db' | head -1)
  echo "items $it"; python3 tools/prof_db.py $db | grep -E "mck|k_link|fold_fast" 
done
