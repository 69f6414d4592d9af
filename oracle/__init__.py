"""ORACLE — CPU restatement of the reference hot path.

TEST INFRASTRUCTURE ONLY.  Nothing in the product (ubpl-poseestimation_amd/)
imports this package; only tests/, __graft_entry__.smoke() and bench.py's
cpu_baseline leg may, and only as the checker / the timed CPU baseline.

Every function cites the reference file:line it restates (paths relative to
the reference root, Qi2019KB/UBPL-PoseEstimation).  The restatement is pinned
against golden vectors produced by running the reference itself in the build
container (tests/golden/gen_golden.py, fixtures tests/golden/*.npz|json);
tests/test_oracle_golden.py is that pin.

Modules
  render    R1   Gaussian heatmap targets           utils/process.py:252-318,393-397
  losses    L1-L7 heatmap/consistency/pseudo/FDL   utils/losses.py, utils/process.py:18-31,381-383, projects/tools.py
  decode    D1-D5 argmax decode, affine back, PCK   utils/udaap/evaluation.py:13-30,215-238, utils/udaap/transforms.py:119-168, utils/evaluation.py:91-139
  schedule  E1-E2 EMA + ramps, S1 sampler           utils/parameters.py, utils/mt/data.py:105-150
  hourglass H1-H6 stacked hourglass (torch CPU fp32)  models/pose/hourglass.py, models/base/layers.py
  step      T1    one training step per project      projects/{MT_UBPL,DualPose_UBPL,MT,supervised}.py
"""
