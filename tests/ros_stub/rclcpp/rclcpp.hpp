#pragma once
#include "ros_stub_all.hpp"
