"""CPU oracle (test infrastructure only).

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s cpu_baseline leg
may import this package, and only as the checker / CPU baseline -- never as the
thing measured or shipped.  The product package ``easywakeword_amd`` must not
import it (enforced by ``tests/test_no_oracle_in_product.py``).
"""
