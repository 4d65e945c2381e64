#!/bin/bash
# Re-make every r06 PMC summary from gpurun_out/prof_* (the final profiling
# calls) on the build host: profiles/r06/rocprof_*_r06.{md,json} and the
# profiles/pmc_*.json records bench.py reads (stamped with the device-code hash)
set -e
cd "$(dirname "$0")/.."
for t in D_512x1M_f153 D_512x1M_f153_i8_certified D_512x1M_f153_i8x2_certified C_1024x131072 B_mnist A_creditcard; do
  python tools/pmc_summary.py gpurun_out/prof_$t $t profiles/r06/rocprof_${t}_r06 10 40 > /dev/null
done
python tools/pmc_summary.py gpurun_out/prof_D_emu8 D_emu8 profiles/r06/rocprof_D_emu8_r06 100 40 > /dev/null
for m in exact mfma certified i8 i8_certified i8x2 i8x2_certified; do
  t=E_4096x262144_fp32; [ "$m" = exact ] || t="${t}_$m"
  python tools/pmc_summary.py gpurun_out/prof_$t $t profiles/r06/rocprof_${t}_r06 5 10 > /dev/null
done
for t in E_emu8_mfma E_emu8_i8x2_certified; do
  python tools/pmc_summary.py gpurun_out/prof_$t $t profiles/r06/rocprof_${t}_r06 20 10 > /dev/null
done
python tools/roni_pmc_summary.py gpurun_out/prof_roni profiles/r06/pmc_roni_r06 > /dev/null
echo summarized
