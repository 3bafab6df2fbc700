"""CPU oracle of the volumetric path — TEST INFRASTRUCTURE ONLY.

A scalar C++ restatement of pbrt-v4's VolPathIntegrator path (volpath_oracle.cpp) and
the recipe that builds the reference's own numerics into oracle/_ref (ref/Makefile).
Imported only by tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg.
"""
