cd "$GRAFT_REPO_ROOT"
export HARNESS_GPU=1 OMPI_AMD_COLL_TIMEOUT_MS=20000 OMPI_AMD_IPC_TRACE=1
for k in 1 2 3; do
  name=$(python3 -c "import secrets;print(secrets.token_hex(3))")
  timeout -k 5 120 tools/pml_harness_bin $name 0 2 > gpurun_out/pml_r0_$k.out 2> gpurun_out/pml_r0_$k.err &
  p0=$!
  timeout -k 5 120 tools/pml_harness_bin $name 1 2 > gpurun_out/pml_r1_$k.out 2> gpurun_out/pml_r1_$k.err
  r1=$?
  wait $p0; r0=$?
  echo "run $k: rc0=$r0 rc1=$r1"
  [ $r0 -eq 0 ] && [ $r1 -eq 0 ] || break
done
