"""Drop-in BO drivers: MultiSurrogateOptimiser, MonoSurrogateOptimiser, EMO, ParEGO, KEEP."""
from .emo import EMO
from .keep import KEEP
from .optimisers import MonoSurrogateOptimiser, MultiSurrogateOptimiser
from .parego import ParEGO

__all__ = ["MultiSurrogateOptimiser", "MonoSurrogateOptimiser", "EMO", "ParEGO", "KEEP"]
