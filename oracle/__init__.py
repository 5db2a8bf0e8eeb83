"""TEST INFRASTRUCTURE ONLY: CPU oracle (checker) for the mgcn hot path.
Imported by tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg;
never by the product package meta-gcn_amd/mgcn."""
