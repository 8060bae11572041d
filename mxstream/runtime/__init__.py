"""mxstream.runtime."""
