#!/bin/bash
# The default bench line on the final in-tree library (engine.hip and migrate.hip memory-clause scheduled).
bash tools/gpu_steps.sh r06zzg "bench|360|python -u bench.py"
