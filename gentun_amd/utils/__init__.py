"""Host utilities: RNG, datasets, fold builders."""
