"""rocket_amd.utils"""
