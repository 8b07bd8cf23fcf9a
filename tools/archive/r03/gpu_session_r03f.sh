cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/c3tl
timeout -s KILL 180 rocprofv3 --kernel-trace -d gpurun_out/c3tl/prof -o run -- python3 -u tools/c3_timeline.py run 256 > gpurun_out/c3tl/run.log 2>&1 || { echo prof failed; tail -20 gpurun_out/c3tl/run.log; exit 1; }
tail -3 gpurun_out/c3tl/run.log
db=$(find gpurun_out/c3tl/prof -name '*.db' | head -1)
echo db=$db
python3 tools/c3_timeline.py show $db > gpurun_out/c3tl/show.txt 2>&1
cat gpurun_out/c3tl/show.txt
