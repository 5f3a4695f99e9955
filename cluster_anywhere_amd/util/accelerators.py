"""Accelerator type constants (reference: util/accelerators/accelerators.py) — the
AMD Instinct family; use as ``@remote(accelerator_type=AMD_INSTINCT_MI355X)``."""
AMD_INSTINCT_MI100 = "AMD-Instinct-MI100"
AMD_INSTINCT_MI210 = "AMD-Instinct-MI210"
AMD_INSTINCT_MI250 = "AMD-Instinct-MI250X-MI250"
AMD_INSTINCT_MI250x = "AMD-Instinct-MI250X-MI250"
AMD_INSTINCT_MI300x = "AMD-Instinct-MI300X-OAM"
AMD_INSTINCT_MI300X = AMD_INSTINCT_MI300x
AMD_INSTINCT_MI325X = "AMD-Instinct-MI325X-OAM"
AMD_INSTINCT_MI350X = "AMD-Instinct-MI350X-OAM"
AMD_INSTINCT_MI355X = "AMD-Instinct-MI355X-OAM"
AMD_RADEON_R9_200_HD_7900 = "AMD-Radeon-R9-200-HD-7900"
AMD_RADEON_HD_7900 = "AMD-Radeon-HD-7900"

__all__ = [n for n in dir() if n.startswith("AMD_")]
