__version__ = "0.1.0"
__reference_version__ = "1.3.0dev"
__license__ = "Apache-2.0"
