cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 200 python -u tools/run_worker.py p2p_osc 2 P2P_OSC_CASES=osc_dynamic_window,osc_accumulate_derived_pair_types,p2p_stage_cap_aged,osc_separate_model_refused TAG=dyn_n > gpurun_out/dyn.log 2>&1; echo rc=$?
cut -c1-600 gpurun_out/dyn.log | tail -8
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_mca_glue.py -k osc > gpurun_out/g.log 2>&1; echo rc=$?
grep -E "FAILED|passed|failed" gpurun_out/g.log | cut -c1-600 | tail -5
