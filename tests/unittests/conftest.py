import pytest

from tests.helpers.ddp import close_pool


@pytest.fixture(scope="session", autouse=True)
def _ddp_pool_teardown():
    yield
    close_pool()
