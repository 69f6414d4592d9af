"""utils/evaluation.py: EvaluationUtils.acc_pck on the HIP path."""
from ubpl_amd.evaluation import EvaluationUtils, final_preds, get_preds  # noqa: F401
