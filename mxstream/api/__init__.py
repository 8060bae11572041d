"""mxstream.api."""
