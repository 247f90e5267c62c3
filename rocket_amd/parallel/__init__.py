"""rocket_amd.parallel"""
