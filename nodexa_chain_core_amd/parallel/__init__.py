"""parallel"""
