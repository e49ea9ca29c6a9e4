"""Reference-compatible `utils` package (utils.utils, utils.data_loader)."""
