S='bash tools/gpu_steps.sh'
O='python -u tools/agent_overhead.py --rate 1e6 --seconds 20'
$S "200|oh_a|$O --out gpurun_out/r5_oh_epi_1.json" \
   "200|oh_b|$O --out gpurun_out/r5_oh_epi_2.json" \
   "200|oh_c|$O --out gpurun_out/r5_oh_epi_3.json" \
   "200|oh_bare|$O --bare --out gpurun_out/r5_oh_epi_bare.json"
