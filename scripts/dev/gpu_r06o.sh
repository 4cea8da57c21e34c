set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r06o
mkdir -p $O
L=transmil_deepgraft_amd
for lib in libtransmil_hip.so libtransmil_hip_g3.so libtransmil_hip_g4.so; do
  TRANSMIL_HIP_LIB=$L/$lib timeout -k 10 300 python -u -m pytest -q -p no:cacheprovider --timeout 120 --timeout-method thread -m gpu \
    tests/test_kernels_gpu.py -k "a3 or sim2" > $O/tests_$lib.txt 2>&1
  rc=$?; echo "$lib: $(tail -1 $O/tests_$lib.txt)"; [ $rc -eq 0 ] || exit $rc
done
for lib in ab/$L/libtransmil_hip.so $L/libtransmil_hip.so $L/libtransmil_hip_g3.so $L/libtransmil_hip_g4.so; do
  echo "== $lib"; TRANSMIL_HIP_LIB=$lib timeout -k 10 120 python scripts/dev/a3_split_time.py 2>&1 | grep -v amdgpu.ids || exit 1
done | tee $O/a3_split_time.txt
echo "== tree A/B: A3 tile init (A) vs HEAD (B)"
AB_PAIRS=3 AB_STEPS=300 bash scripts/dev/ab_tree.sh run 2>&1 | tee $O/ab_a3_init.txt
