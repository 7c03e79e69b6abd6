"""CPU parity oracle — TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import
this package, and only as the checker / CPU baseline; the product package
(qldpcsim_amd) never imports, links or executes anything under oracle/.
"""
