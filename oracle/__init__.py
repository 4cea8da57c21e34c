"""CPU oracle for the TransMIL forward/backward hot path.

TEST INFRASTRUCTURE ONLY -- the checker, never the thing measured or shipped.
Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s
``cpu_baseline`` leg may import anything from here.

* ``nystrom_ref``  -- restatement of the third-party ``nystrom_attention``
  (not vendored by the reference; parity of its internals UNPINNED, see
  DESIGN.md section 3).
* ``transmil_ref`` -- restatement of ``code/models/TransMIL.py`` (pinned by
  the golden fixtures made by importing the reference itself).
"""
