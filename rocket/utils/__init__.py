"""``rocket.utils`` (reference ``rocket/utils``) backed by :mod:`rocket_amd.utils`."""
