"""Replay only the dominant kernel of the step (fqlpop_dominant_kernel_info:
the persistent Euler flow at H = 512, 16 members in one launch) for PMC
collection under rocprofv3 (developer tool):

  rocprofv3 --pmc FETCH_SIZE --kernel-include-regex euler_flow -- python3 profile_dominant.py
"""
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))

from fqlpop import Population, PopulationConfig  # noqa: E402

pop = Population(PopulationConfig(), [10.0] * 16, list(range(16)))
us, flops = pop.time_dominant_kernel(int(sys.argv[1]) if len(sys.argv) > 1 else 20)
print(f"dominant kernel {pop.dominant_kernel_info()[0]}: {us:.2f} us/launch, {flops / 1e9:.3f} GFLOP/launch")
