#!/bin/bash
# Final evidence on the engine built with memory-clause scheduling (keto_amd/build.py SOURCE_FLAGS):
# the full -m gpu suite, smoke, bench, rocprofv3 kernel trace and the two PMC traffic passes.
bash tools/gpu_round.sh r06zzd
