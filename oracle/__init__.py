"""CPU oracle for the batched BFGS bundle-adjustment hot path.

TEST INFRASTRUCTURE ONLY.  Nothing in the product package
(``deep-attention-visual-odometry_amd/``) imports, links or executes this
package.  Only ``tests/``, ``__graft_entry__.smoke()`` and the
``cpu_baseline`` leg of ``bench.py`` may use it, and only as the checker /
CPU baseline, never as the thing measured or shipped.

It is a PyTorch-CPU restatement of the reference algorithm
(jskinn/deep-attention-visual-odometry @ 2025-04-04):

* ``oracle.trig``       -- Taylor-branched trig ratios with their custom
                           backward formulas (``utils/func_sin_x_on_x.py``,
                           ``utils/func_one_minus_cos_x_on_x_squared.py``).
* ``oracle.objective``  -- multi-view pinhole (+ Brown-Conrady) squared
                           reprojection error (``camera_model/`` +
                           ``geometry/``), SURVEY.md section 8(a).
* ``oracle.solver``     -- eval-mode ``BFGSSolver.forward`` and the strong
                           Wolfe line search (``autograd_solvers/``).

Parity pinning: ``tests/golden/make_golden.py`` imports the reference from
``/root/reference`` (build container only) and writes golden vectors to
``tests/golden/*.npz``; ``tests/test_oracle_golden.py`` checks this oracle
against them bit-for-bit (fp64) / within 1e-6 normwise (fp32).  The
Brown-Conrady block has no runnable reference (its module imports the absent
``spatial_maths`` package), so that part is pinned only by restatement of
``camera_model/distorted_camera_model.py:59-86`` plus autograd/finite-difference
checks -- "parity unpinned" for distortion, see DESIGN.md.
"""
