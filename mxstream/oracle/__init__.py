"""mxstream.oracle."""
