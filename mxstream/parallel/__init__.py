"""mxstream.parallel."""
