cd $GRAFT_REPO_ROOT
TAG=rd1 bash tools/gpu_tests.sh || exit 1
TAG=abw10 TESTS=none WORKLOADS="cfg2 cfg5 cfg3" bash tools/ab_workloads.sh
