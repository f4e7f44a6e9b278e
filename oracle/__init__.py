"""ORACLE — test infrastructure only.

CPU restatement of the reference (tanwanirahul/surreal) learner hot path, used
ONLY as the checker by tests/, __graft_entry__.smoke() and bench.py's
cpu_baseline leg.  Nothing in surreal_amd/ imports it; the product path never
routes through it.

Pinning: running or importing the reference in this environment was denied
(SURVEY.md §8(c)), and the reference holds no golden vectors or numeric tests
for this path.  The restatement is therefore pinned by:
  * hand-derived known answers committed under tests/golden/ (closed forms for
    GAE, DiagGauss, ZFilter, Adam, clip loss), and
  * CPython stdlib `random` index streams for the uniform replay sampler (the
    reference calls random.randint directly), which pin the MT19937 restatement
    bit-exactly.
Everything else is "parity partially pinned": the floating-point learner math
follows the cited reference lines op by op, in fp32 on the CPU.
"""
