"""utils/parameters.py: flat-buffer EMA on the HIP path + the ramps."""
from ubpl_amd.parameters import (FDLWeight_decrease, FDLWeight_increase, _sigmoid_rampup,  # noqa: F401
                                 _value_decrease, _value_increase, consWeight_increase,
                                 pseudoWeight_increase, update_ema_variables)
