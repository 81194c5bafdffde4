# Repeats the 3-rank osc component device-path test under a few env
# settings; one line per config: passes / failures and the first mismatch.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/oscflake
for cfg in ${CFGS:-BASE=1 OMPI_AMD_DDT_TILE=0 OMPI_AMD_OSC_MAX_BLOCKS=1}; do
  ok=0; bad=0; first=""
  for i in $(seq 1 ${REPS:-12}); do
    env $cfg timeout -k 10 120 python -u -m pytest -x -q --timeout 100 --timeout-method thread -m gpu \
      tests/test_mca_glue.py -k "osc_component_device_path and 3" > gpurun_out/oscflake/run.log 2>&1
    rc=$?
    if [ $rc -eq 0 ]; then ok=$((ok+1)); else
      bad=$((bad+1)); [ -z "$first" ] && first=$(grep -h "derived get:" gpurun_out/oscflake/run.log | head -1 | cut -c1-200)
      cp gpurun_out/oscflake/run.log gpurun_out/oscflake/fail_${cfg%%=*}_$i.log
      [ $rc -ge 124 ] && { echo "$cfg: timeout rc $rc, stop"; exit 1; }
    fi
  done
  echo "$cfg: ok $ok bad $bad $first"
done
