"""TEST INFRASTRUCTURE ONLY -- the CPU checkers for the team::Align path.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may
import this package.  The product (bioinfo1_amd, libteam_alignment.so) never
does.
"""
