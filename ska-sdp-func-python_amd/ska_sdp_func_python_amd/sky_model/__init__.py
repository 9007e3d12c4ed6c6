"""Sky-model predict / invert drivers over the hot path."""
from .skymodel_imaging import skymodel_calibrate_invert, skymodel_predict_calibrate  # noqa: F401
