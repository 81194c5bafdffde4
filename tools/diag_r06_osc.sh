#!/bin/bash
# Round-6 diagnostic of the separate-model osc mismatch.
# Each step: rc 0 (green) or 1 (parity failure) continues; anything else stops.
cd "$(dirname "$0")/.." || exit 2
out=gpurun_out/diag
mkdir -p $out
step() {
  local name=$1; shift
  echo "== $name $(date +%T)"
  timeout -k 10 280 python -u tools/run_worker.py "$@" TAG=${name}_n > $out/$name.log 2>&1
  local rc=$?
  grep -h "DIAG" gpurun_out/coll_logs/raw_${name}_n*_rank*.txt | head -40
  tail -2 $out/$name.log | cut -c1-400
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "STOP rc=$rc"; exit $rc; fi
}
H=p2p_random_channels,p2p_random_channels_b,p2p_random_channels_any_source
for spec in "$@"; do
  case $spec in
    force3000) step force3000 p2p_osc 8 P2P_OSC_CASES=osc_random_epochs OSC_DIAG=1 STRESS_SEED=3000 OSC_FORCE_SHADOW=1 ;;
    force0) step force0 p2p_osc 8 P2P_OSC_CASES=osc_random_epochs OSC_DIAG=1 STRESS_SEED=0 OSC_FORCE_SHADOW=1 ;;
    hist3000) step hist3000 p2p_osc 8 P2P_OSC_CASES=$H,osc_random_epochs OSC_DIAG=1 STRESS_SEED=3000 ;;
    hist5000) step hist5000 p2p_osc 8 P2P_OSC_CASES=$H,osc_random_epochs OSC_DIAG=1 STRESS_SEED=5000 ;;
    hist3000_eager) step hist3000_eager p2p_osc 8 P2P_OSC_CASES=$H,osc_random_epochs OSC_DIAG=1 STRESS_SEED=3000 OMPI_AMD_EAGER_CLOSE_MARK=1 ;;
    hist5000_eager) step hist5000_eager p2p_osc 8 P2P_OSC_CASES=$H,osc_random_epochs OSC_DIAG=1 STRESS_SEED=5000 OMPI_AMD_EAGER_CLOSE_MARK=1 ;;
    end3000) step end3000 p2p_osc 8 P2P_OSC_CASES=$H,osc_random_epochs OSC_DIAG=2 STRESS_SEED=3000 ;;
    end5000) step end5000 p2p_osc 8 P2P_OSC_CASES=$H,osc_random_epochs OSC_DIAG=2 STRESS_SEED=5000 ;;
    endforce3000) step endforce3000 p2p_osc 8 P2P_OSC_CASES=osc_random_epochs OSC_DIAG=2 STRESS_SEED=3000 OSC_FORCE_SHADOW=1 ;;
    endforce5000) step endforce5000 p2p_osc 8 P2P_OSC_CASES=osc_random_epochs OSC_DIAG=2 STRESS_SEED=5000 OSC_FORCE_SHADOW=1 ;;
    plain3000) step plain3000 p2p_osc 8 P2P_OSC_CASES=$H,osc_random_epochs STRESS_SEED=3000 ;;
    plain3000_eager) step plain3000_eager p2p_osc 8 P2P_OSC_CASES=$H,osc_random_epochs STRESS_SEED=3000 OMPI_AMD_EAGER_CLOSE_MARK=1 ;;
  esac
done
