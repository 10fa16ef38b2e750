from gsvc_amd.version import __version__  # noqa: F401
