"""Linear-probe evaluation of trained students (reference `tools/lineval/`)."""
