bash scripts/gpu_iter.sh && NO_PMC=1 bash scripts/gpu_prof.sh r01b
