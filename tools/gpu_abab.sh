# Alternating A/B bench of two builds of the same ABI: A = learningagileflight_se3_amd/liblafse3_A.so,
# B = the in-tree liblafse3.so; four quick bench runs each, interleaved (clock / thermal drift cancels).
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
: > gpurun_out/abab.log
for i in 1 2 3; do
  LAFSE3_LIB=$GRAFT_REPO_ROOT/learningagileflight_se3_amd/liblafse3_A.so timeout -k 10 200 python bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-extra | sed 's/^/A /' >> gpurun_out/abab.log || exit $?
  timeout -k 10 200 python bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-extra | sed 's/^/B /' >> gpurun_out/abab.log || exit $?
done
