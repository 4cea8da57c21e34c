"""Drop-in for the reference plugin package ``models`` (ModelInterface.load_model
imports ``models.{name}`` and fetches the class of the same name,
code/models/model_interface.py:1256-1276)."""
from .TransMIL import TransMIL, TransLayer, PPEG  # noqa: F401
from .MDMIL import MDMIL  # noqa: F401
from .CTMIL import CTMIL  # noqa: F401
from .TransformerMIL import TransformerMIL  # noqa: F401
from .AttMIL import AttMIL  # noqa: F401
