mkdir -p gpurun_out
bash scripts/gpu_steps.sh smoke tests_all bench prof pmc
