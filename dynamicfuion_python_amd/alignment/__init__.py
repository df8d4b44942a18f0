"""Mirror of the reference's Python `alignment` package slot on the fitter path (alignment/render_based)."""
