"""Oracle package -- TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import
this package.  The product (nip_amd/) never does.

* ``oracle.bind.PortOracle``  -- the standalone C restatement (nip_oracle.c)
* ``oracle.bind.RefHarness``  -- the reference's own code (oracle/_ref), only
  where it was built (this container, or a snapshot carrying the built .so)
* ``oracle.netfile``          -- a small independent Hugin .net reader
"""
