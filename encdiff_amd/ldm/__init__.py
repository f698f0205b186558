"""Mirror of the reference ``ldm`` package API for the EncDiff denoising path."""
