set -o pipefail
bash tools/prof.sh r02e_c2 --config c2 || exit 1
bash tools/prof.sh r02e_c2_volume --config c2 --path volume || exit 1
bash tools/prof.sh r02e_c4 --config c4 || exit 1
timeout -k 10 200 python tools/post_bench.py --configs c4 c2 c5 > gpurun_out/r02e_post_bench.jsonl || exit 1
cd /tmp && export TMPDIR=/tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/prof_r02e_post/trace -o run -- python3 $GRAFT_REPO_ROOT/tools/post_bench.py --configs c4 --runs 50 > /dev/null || exit 1
