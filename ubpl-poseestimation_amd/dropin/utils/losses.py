"""utils/losses.py on the HIP path (JointMSELoss, JointDistLoss, JointDistLoss_mt2,
JointPseudoLoss3, JointFeatureDistLoss, AvgCounter, AvgCounters)."""
from ubpl_amd.losses import (AvgCounter, AvgCounters, JointDistLoss, JointDistLoss_mt2,  # noqa: F401
                             JointFeatureDistLoss, JointMSELoss, JointPseudoLoss3)
