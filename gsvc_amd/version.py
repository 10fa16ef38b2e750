"""Version of the gsvc_amd drop-in (API level: gsplat 0.1.3 as vendored by GSVC)."""
__version__ = "0.1.3+gsvc_amd.1"
